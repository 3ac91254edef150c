"""Build libsmi_amd.so in-tree with hipcc for gfx950.

The library is the drop-in C ABI declared in include/smi/*.h: hand-written
HIP kernels (csrc/*.hip) plus the native runtime (csrc/*.cpp, RCCL
transport).  Built here with no GPU present (hipcc cross-compiles) and
shipped in-tree to the GPU box.
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libsmi_amd.so")
ARCH = os.environ.get("SMI_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

# -ffp-contract=off: HIP defaults to fast contraction; every kernel here has
# a fixed fp32 evaluation order that an FMA would change (stencil_smi.cl:
# 153-156, reduce.cl:65-125, gesummv_rank0.cl:137-171).
CXXFLAGS = [
    "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
    f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
    f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}",
]
# Per-file extras (by file-name prefix).  The K-step sweeps (stencilk.h /
# stencild.h, instantiated in stencilk_k<K>.hip / stencild_k<K>.hip) spell
# out which adds are packed (v_pk_add_f32 on aligned pairs); the SLP
# vectorizer would pack the shuffled (S+W)/(+E) adds too and pay a register
# move for each pair (the rotating-ring sweep ran 0.217 instead of ~0.15 ms
# per K = 20 pass without this flag).
FILE_FLAGS = {"stencilk_k": ["-fno-slp-vectorize"], "stencild_k": ["-fno-slp-vectorize"],
              "bandk_k": ["-fno-slp-vectorize"]}
# Build variants, each in its own directory: the product library (no
# experiment switch is compiled into it), a bounds-checked diagnostic build,
# the loopback rehearsal build (tools/rehearsal.py: SMI_LOOPBACK* switches)
# and the experiment build (SMI_FOLD_VARIANT / SMI_GEMV_VARIANT launch
# variants read from the environment).
VARIANT_FLAGS = {
    "": [],
    "debug": ["-DSMI_BOUNDS_CHECK"],
    "rehearsal": ["-DSMI_LOOPBACK_REHEARSAL"],
    "experiments": ["-DSMI_EXPERIMENTS"],
}


# Sources no variant switch reaches (no SMI_LOOPBACK* / SMI_BOUNDS_CHECK /
# SMI_EXPERIMENTS in them or in what they include): every variant links the
# release objects of these instead of compiling them again (the rotating-ring
# sweep's eight instantiation units take minutes each; the K-step sweeps'
# and the band kernels' too).
SHARED_PREFIXES = ("stencild_k", "stencilk_k", "bandk_k")


def file_flags(src: str) -> list[str]:
    name = os.path.basename(src)
    return [f for prefix, fl in FILE_FLAGS.items() if name.startswith(prefix) for f in fl]
LDFLAGS = ["-shared", f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]


def sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def lib_path(variant: str = "") -> str:
    """release: _build/libsmi_amd.so; otherwise _build/<variant>/libsmi_amd_<variant>.so."""
    if not variant:
        return LIB
    if variant not in VARIANT_FLAGS:
        raise ValueError(f"unknown build variant {variant!r}")
    return os.path.join(OUT_DIR, variant, f"libsmi_amd_{variant}.so")


def _lib_deps() -> list[str]:
    return sorted(sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(
        os.path.join(ROOT, "include", "**", "*.h"), recursive=True))


def _src_hash(variant: str = "") -> str:
    """Content hash of every source and header the library is built from,
    with the build flags."""
    import hashlib
    h = hashlib.sha256()
    flags = " ".join(CXXFLAGS + VARIANT_FLAGS[variant] + [f"{k}={v}" for k, v in sorted(FILE_FLAGS.items())])
    h.update(flags.replace(ROOT, "<root>").encode())  # the same tree anywhere on disk
    for d in _lib_deps():
        h.update(os.path.relpath(d, ROOT).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale(variant: str = "") -> bool:
    """The library is stale when a source or header is newer than it AND the
    sources' content differs from what it was built from (a copied tree --
    the GPU box's snapshot, a checkout -- may carry newer mtimes for the same
    content: rebuilding there would take many minutes for nothing)."""
    lib = lib_path(variant)
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    if not any(os.path.getmtime(d) > t for d in _lib_deps()):
        return False
    try:
        with open(lib + ".srchash") as f:
            return f.read().strip() != _src_hash(variant)
    except OSError:
        return True


def _deps(src: str, seen: set | None = None) -> set:
    """src and every header it includes with "..." (recursively), resolved
    against its directory, csrc/ and include/."""
    import re
    seen = set() if seen is None else seen
    if src in seen or not os.path.exists(src):
        return seen
    seen.add(src)
    with open(src, errors="replace") as f:
        for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
            for d in (os.path.dirname(src), CSRC, os.path.join(ROOT, "include")):
                cand = os.path.join(d, inc)
                if os.path.exists(cand):
                    _deps(cand, seen)
                    break
    return seen


def _obj_stale(src: str, obj: str, flags_file: str) -> bool:
    if not os.path.exists(obj) or not os.path.exists(flags_file):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in _deps(src) | {flags_file})


def build(force: bool = False, verbose: bool = False, variant: str = "") -> str:
    lib = lib_path(variant)
    if not force and not _stale(variant):
        return lib
    out_dir = os.path.dirname(lib)
    os.makedirs(out_dir, exist_ok=True)
    flags = CXXFLAGS + VARIANT_FLAGS[variant]
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    # objects are rebuilt when their source, a header they include or the
    # flags changed (the flags are recorded next to the objects)
    flags_file = os.path.join(out_dir, "flags.txt")
    flags_txt = " ".join(flags + [f"{k}={v}" for k, v in sorted(FILE_FLAGS.items())])
    if not os.path.exists(flags_file) or open(flags_file).read() != flags_txt:
        with open(flags_file, "w") as f:
            f.write(flags_txt)
    objs = []
    procs = []
    if variant:
        shared = [src for src in sources() if os.path.basename(src).startswith(SHARED_PREFIXES)]
        if shared:
            build(force=force, verbose=verbose)  # the release objects they come from
    for src in sources():
        if variant and os.path.basename(src).startswith(SHARED_PREFIXES):
            objs.append(os.path.join(OUT_DIR, os.path.basename(src) + ".o"))
            continue
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if not force and not _obj_stale(src, obj, flags_file):
            continue
        cmd = [hipcc, *flags, *file_flags(src), "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((src, out.decode(errors="replace")))
        elif verbose and out:
            print(out.decode(errors="replace"), file=sys.stderr)
    if failed:
        msg = "\n".join(f"--- {s}\n{o}" for s, o in failed)
        raise RuntimeError(f"hipcc failed:\n{msg}")
    tmp = lib + ".tmp"
    subprocess.run([hipcc, *objs, *LDFLAGS, f"--offload-arch={ARCH}", "-o", tmp], check=True)
    os.replace(tmp, lib)
    with open(lib + ".srchash", "w") as f:
        f.write(_src_hash(variant) + "\n")
    return lib


HOSTS_DIR = os.path.join(ROOT, "hosts")


def build_hosts(force: bool = False, verbose: bool = False) -> list[str]:
    """Compile the C++ host programs (hosts/*.cpp: the reference host programs
    restated on the C ABI) against include/ and the release libsmi_amd.so into
    hosts/_build/, linked with an $ORIGIN-relative rpath so they run from any
    copy of the tree (the GPU box's snapshot included)."""
    lib = build()
    out_dir = os.path.join(HOSTS_DIR, "_build")
    os.makedirs(out_dir, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    outs = []
    # a host is fresh when the content hash of its source, the hosts'
    # shared headers, include/ and the library's own source hash matches the
    # one recorded beside it (mtimes mislead on a copied tree)
    common = sorted(glob.glob(os.path.join(HOSTS_DIR, "*.h")) + glob.glob(
        os.path.join(ROOT, "include", "**", "*.h"), recursive=True))
    with open(lib + ".srchash") as f:
        lib_hash = f.read().strip()
    for src in sorted(glob.glob(os.path.join(HOSTS_DIR, "*.cpp"))):
        exe = os.path.join(out_dir, os.path.splitext(os.path.basename(src))[0])
        outs.append(exe)
        cmd = [hipcc, "-O2", "-std=c++17", "-Wall", f"--offload-arch={ARCH}", f"-I{os.path.join(ROOT, 'include')}",
               src, "-o", exe,
               f"-L{OUT_DIR}", "-lsmi_amd", "-lpthread", "-Wl,-rpath,$ORIGIN/../../smi_amd/_build",
               f"-Wl,-rpath,{ROCM}/lib"]
        h = hashlib.sha256(lib_hash.encode())
        for p in [src] + common:
            with open(p, "rb") as f:
                h.update(os.path.relpath(p, ROOT).encode() + b"\0" + f.read())
        h.update(" ".join(cmd).replace(ROOT, "<root>").encode())
        digest = h.hexdigest()
        stamp = exe + ".srchash"
        if not force and os.path.exists(exe) and os.path.exists(stamp):
            with open(stamp) as f:
                if f.read().strip() == digest:
                    continue
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        with open(stamp, "w") as f:
            f.write(digest + "\n")
    return outs


if __name__ == "__main__":
    if "--hosts" in sys.argv:
        print("\n".join(build_hosts(force="--force" in sys.argv, verbose=True)))
        sys.exit(0)
    v = next((a[2:] for a in sys.argv[1:] if a.startswith("--") and a[2:] in VARIANT_FLAGS), "")
    print(build(force="--force" in sys.argv, verbose=True, variant=v))
