#!/usr/bin/env python3
"""Resource footprint of the RCCL kernels libsmi_amd.so binds to, beside ours.

The halo exchange of a multi-rank pass is an RCCL group (ncclSend/ncclRecv,
transport.cpp) whose kernel must find wave slots on CUs where the interior
sweep (sweepd_kernel<K>) already holds two waves per SIMD.  This tool reads
the gfx950 kernel descriptors of

  * the librccl.so that libsmi_amd.so actually resolves to once torch is
    imported (smi_amd/_lib.py loads torch first, so its bundled copy wins;
    found through /proc/self/maps after loading the library), and
  * our own kernels (sweepd_kernel<K>, bandl/bandk_kernel<K>) from the
    objects in smi_amd/_build,

and prints the VGPR / AGPR / LDS / workgroup-size figures plus whether one
RCCL workgroup fits on a CU beside the interior's resident waves: a SIMD has
512 unified registers per lane, allocated in granules of 8.

    python tools/rccl_footprint.py [--json profiles/r05/rccl_footprint.json]

Runs on the build host (no GPU needed: HIP is never initialised).
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LLVM = "/opt/rocm/lib/llvm/bin"
ARCH = "gfx950"
SIMD_REGS = 512     # unified VGPR + AGPR file per lane and SIMD (MI355X_MICROARCH.md)
GRANULE = 8         # allocation granule (wave64)


def bound_rccl() -> str:
    """Path of the librccl the process maps after import torch + our library."""
    import ctypes

    import torch  # noqa: F401  (the same load order as smi_amd/_lib.py)
    from smi_amd import build
    ctypes.CDLL(build.lib_path(), mode=ctypes.RTLD_GLOBAL)
    with open("/proc/self/maps") as f:
        for line in f:
            if "librccl" in line:
                return os.path.realpath(line.split()[-1])
    raise RuntimeError("no librccl mapped")


def code_object(path: str, tmp: str) -> str:
    fat = os.path.join(tmp, os.path.basename(path) + ".fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path,
                    os.path.join(tmp, "discard.o")], check=True)
    listed = subprocess.run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={fat}"],
                            check=True, capture_output=True, text=True).stdout.split()
    target = next(t for t in listed if t.endswith("--" + ARCH) or ("--" + ARCH + ":") in t)
    co = os.path.join(tmp, os.path.basename(path) + ".co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets={target}", f"--output={co}"], check=True)
    os.unlink(fat)
    return co


def kernels(co: str, pattern: str) -> list[dict]:
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    out = []
    # one YAML map per kernel under amdhsa.kernels: split on the list dashes
    for blk in re.split(r"\n\s+- \.", notes):
        m = re.search(r"\.?name:\s+(\S+)", blk)
        if not m or not re.search(pattern, m.group(1)) or ".symbol:" not in blk:
            continue
        ent = {"symbol": m.group(1)}
        for key in ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size",
                    "max_flat_workgroup_size", "private_segment_fixed_size", "vgpr_spill_count",
                    "sgpr_spill_count"):
            mm = re.search(r"\." + key + r":\s+(\d+)", blk)
            if mm:
                ent[key] = int(mm.group(1))
        # .vgpr_count on gfx90a+ is the unified allocation (arch VGPRs aligned
        # to 4, then the AGPRs) -- what occupancy is computed from
        ent["regs_per_lane"] = -(-ent.get("vgpr_count", 0) // GRANULE) * GRANULE
        out.append(ent)
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    ap.add_argument("--k", type=int, default=20)
    a = ap.parse_args()
    rccl = bound_rccl()
    res = {"librccl": rccl, "arch": ARCH, "simd_regs_per_lane": SIMD_REGS, "granule": GRANULE}
    with tempfile.TemporaryDirectory(prefix="rccl_fp_") as tmp:
        rk = kernels(code_object(rccl, tmp), r"rcclGenericKernel")
        ours = []
        for obj, pat in ((f"stencild_k{a.k}.hip.o", rf"sweepd_kernelILi{a.k}E"),
                         (f"bandk_k{a.k}.hip.o", rf"band[kl]_kernelILi{a.k}E")):
            ours += kernels(code_object(os.path.join(ROOT, "smi_amd", "_build", obj), tmp), pat)
    for lst in (rk, ours):
        for e, d in zip(lst, demangle([e["symbol"] for e in lst])):
            e["kernel"] = d
    res["rccl_kernels"] = rk
    res["our_kernels"] = ours
    interior = next(e for e in ours if "sweepd" in e["symbol"])
    waves = SIMD_REGS // interior["regs_per_lane"]
    free = SIMD_REGS - waves * interior["regs_per_lane"]
    res["interior"] = {"kernel": interior["kernel"], "regs_per_lane": interior["regs_per_lane"],
                       "waves_per_simd": waves, "free_regs_per_simd_when_resident": free}
    res["coresidency"] = [
        {"kernel": e["kernel"], "regs_per_lane": e["regs_per_lane"],
         "fits_beside_full_interior": e["regs_per_lane"] <= free,
         "fits_beside_one_interior_wave": e["regs_per_lane"] <= SIMD_REGS - interior["regs_per_lane"],
         "waves_per_workgroup": e.get("max_flat_workgroup_size", 0) // 64,
         "lds_bytes": e.get("group_segment_fixed_size")}
        for e in rk + [o for o in ours if "sweepd" not in o["symbol"]]]
    print(json.dumps(res, indent=1))
    if a.json:
        os.makedirs(os.path.dirname(os.path.abspath(a.json)), exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
