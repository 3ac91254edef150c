"""The drop-in boundary on CPU: libsmi_amd.so builds for gfx950, loads, and
exports every function include/smi/*.h declares (no compute without a GPU)."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECL = re.compile(r"^\s*(?:const\s+)?[A-Za-z_]\w*\s*\**\s*((?:smi|SMI)_\w+)\s*\(", re.M)


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "**", "*.h"), recursive=True):
        text = open(h).read()
        text = re.sub(r"static inline[^{]*\{[^}]*\}", "", text)  # header-only helpers
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)  # comments
        syms.update(DECL.findall(text))
    return sorted(syms)


@pytest.fixture(scope="module")
def lib():
    from smi_amd import _lib
    return _lib.load()


def test_headers_declare_the_surface():
    syms = declared_symbols()
    for must in ("smi_init", "smi_finalize", "smi_stencil_run", "smi_stencil_step", "smi_reduce", "smi_bcast",
                 "smi_gesummv", "smi_gemv_rows", "smi_reduce_fold", "smi_get_unique_id", "SMI_Push", "SMI_Pop",
                 "SMI_Open_send_channel", "SMI_Bcast", "SMI_Reduce", "SMI_Scatter", "SMI_Gather", "smi_scatter"):
        assert must in syms


def test_every_declared_symbol_is_exported(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_every_symbol():
    from smi_amd import _lib
    assert set(declared_symbols()) <= set(_lib.SIGNATURES)


def test_library_is_gfx950_code_object(lib):
    from smi_amd import _lib
    data = open(_lib.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # the embedded offload bundle id
    assert b"gfx942" not in data and b"gfx90a" not in data


def test_calls_without_gpu_fail_loudly(lib):
    """No GPU here: entry points that need one return an error code (and the
    Python mirror raises) instead of silently computing on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from smi_amd import SMIError, _lib
    c = _lib.SMI_Comm()
    rc = lib.smi_init_local(1, 0, 0, ctypes.byref(c))
    assert rc != 0
    with pytest.raises(SMIError):
        _lib.call("smi_init_local", 1, 0, 0, ctypes.byref(c))
    n = ctypes.c_int(-1)
    assert lib.smi_device_count(ctypes.byref(n)) == 0 and n.value == 0


def test_enum_values_match_reference():
    """Same enumerators and values as the reference headers
    (include/smi/data_types.h:10-16, reduce.h:18-22, operation_type.h:11-19)."""
    text = "".join(open(p).read() for p in glob.glob(os.path.join(ROOT, "include", "smi", "*.h")))
    for name, val in [("SMI_INT", 1), ("SMI_FLOAT", 2), ("SMI_DOUBLE", 3), ("SMI_CHAR", 4), ("SMI_SHORT", 5),
                      ("SMI_ADD", 0), ("SMI_MAX", 1), ("SMI_MIN", 2), ("SMI_SEND", 0), ("SMI_RECEIVE", 1),
                      ("SMI_BROADCAST", 2), ("SMI_SYNCH", 3), ("SMI_SCATTER", 4), ("SMI_REDUCE", 5),
                      ("SMI_GATHER", 6)]:
        assert re.search(rf"\b{name}\s*=\s*{val}\b", text), name


def test_c_header_compiles_standalone(tmp_path):
    """A C host program (the reference hosts are C/C++) can include smi.h and
    link against the library."""
    src = tmp_path / "t.c"
    src.write_text('#include "smi.h"\n#include <stdio.h>\nint main(void){int n=0;'
                   'smi_device_count(&n);SMI_Comm c={0,1,0};printf("%d %d\\n",SMI_Comm_size(c),n);'
                   'return 0;}\n')
    from smi_amd import _lib
    libdir = os.path.dirname(_lib.lib_path())
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", f"-I{ROOT}/include", str(src), "-o", str(exe),
                    f"-L{libdir}", "-lsmi_amd", f"-Wl,-rpath,{libdir}"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True)
    assert out.stdout.split()[0] == "1"


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A library whose recorded source hash differs from this tree's is never
    loaded: a copy with a tampered .srchash raises, on a
    GPU host and on the build host alike (the mtimes say "fresh", so nothing
    rebuilds it), and the untampered copy passes."""
    import shutil

    from smi_amd import _lib
    src = _lib.lib_path()
    _lib.load()  # the real library is fresh
    dst = tmp_path / "libsmi_amd.so"
    shutil.copy(src, dst)
    shutil.copy(src + ".srchash", str(dst) + ".srchash")
    assert _lib.verify_fresh(str(dst)) == _lib._build._src_hash()
    (tmp_path / "libsmi_amd.so.srchash").write_text("0" * 64 + "\n")
    with pytest.raises(_lib.SMIError, match="not built from these sources"):
        _lib.verify_fresh(str(dst))
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "lib_path", lambda: str(dst))
    for bim in (False, True):
        with pytest.raises(_lib.SMIError, match="not built from these sources"):
            _lib.load(build_if_missing=bim)
    (tmp_path / "libsmi_amd.so.srchash").unlink()
    with pytest.raises(_lib.SMIError, match="missing"):
        _lib.load(build_if_missing=False)
