#!/usr/bin/env python3
"""Instruction histogram of a kernel's steady-state loops from its gfx950 ISA.

Extracts the gfx950 code object from a hipcc object file (the `.hip_fatbin`
section, `clang-offload-bundler`), disassembles it with `llvm-objdump`, finds
every loop of the named kernel (a branch whose target lies before it) and
prints, per loop, the instruction classes of its body: plain VALU adds,
packed adds, DPP moves / DPP-fused adds, cndmask, frexp / min / max,
readlane / writelane (SGPR spills), vector loads and stores, scalar
instructions and waits.  With --per N each count is also divided by N
(e.g. the loop body's rows x levels) for per-row figures.

    python tools/isa_hist.py smi_amd/_build/stencild_k20.hip.o \
        --kernel sweepd_kernelILi20E --rows 44 --levels 20 --json out.json
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ADDR = re.compile(r"//\s*([0-9A-Fa-f]{12,16}):")
TARGET = re.compile(r"<([^>+]*)\+0x([0-9a-f]+)>")


def disassemble(obj, arch="gfx950"):
    tmp = tempfile.mkdtemp(prefix="isa_hist_")
    fat = os.path.join(tmp, "fat.bin")
    co = os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(tmp, "o")],
                   check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets=hipv4-amdgcn-amd-amdhsa--{arch}", f"--output={co}"], check=True)
    asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                         check=True, capture_output=True, text=True).stdout
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    return asm, notes


def kernel_lines(asm, kernel):
    """[(offset_in_kernel, mnemonic, text)] of the first symbol containing `kernel`."""
    out, cur, base = [], None, None
    for line in asm.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            cur = m.group(2)
            base = int(m.group(1), 16)
            continue
        if cur is None or kernel not in cur:
            if out:
                break
            continue
        a = ADDR.search(line)
        if not a:
            continue
        text = line.split("//")[0].strip()
        if not text:
            continue
        t = TARGET.search(line)
        if t:
            text += " <+0x" + t.group(2) + ">"
        out.append((int(a.group(1), 16) - base, text.split()[0], text))
    return out


def classify(mn, text):
    if mn.startswith("v_"):
        dpp = "row_" in text or "wave_" in text or "quad_perm" in text or "row_shr" in text
        if mn in ("v_readlane_b32", "v_writelane_b32", "v_readfirstlane_b32"):
            return "valu_lane(" + mn + ")"
        if mn.startswith("v_pk_add_f32"):
            return "valu_pk_add_f32"
        if mn.startswith("v_pk_mul_f32"):
            return "valu_pk_mul_f32"
        if mn.startswith("v_add_f32"):
            return "valu_add_f32_dpp" if dpp else "valu_add_f32"
        if mn.startswith("v_mov_b32"):
            return "valu_mov_dpp" if dpp else "valu_mov"
        if mn.startswith("v_cndmask"):
            return "valu_cndmask"
        if "frexp" in mn:
            return "valu_frexp"
        if mn.startswith(("v_min", "v_max")):
            return "valu_minmax"
        return "valu_other(" + mn + ")"
    if mn.startswith(("global_load", "buffer_load")):
        return "vmem_load"
    if mn.startswith(("global_store", "buffer_store")):
        return "vmem_store"
    if mn.startswith("s_waitcnt"):
        return "s_waitcnt"
    if mn.startswith("s_nop"):
        return "s_nop"
    if mn.startswith(("s_branch", "s_cbranch")):
        return "s_branch"
    if mn.startswith("s_"):
        return "salu/smem"
    return "other(" + mn + ")"


def loops(lines):
    """Loops as (start_index, end_index) from backward branches."""
    idx = {off: i for i, (off, _, _) in enumerate(lines)}
    res = []
    for i, (off, mn, text) in enumerate(lines):
        if not mn.startswith(("s_branch", "s_cbranch")):
            continue
        t = TARGET.search(text)
        if not t:
            continue
        tgt = int(t.group(2), 16)
        if tgt < off and tgt in idx:
            res.append((idx[tgt], i))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("obj")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--rows", type=int, default=0, help="input rows per loop body")
    ap.add_argument("--levels", type=int, default=0, help="levels per input row")
    ap.add_argument("--json")
    a = ap.parse_args()
    asm, notes = disassemble(a.obj)
    lines = kernel_lines(asm, a.kernel)
    if not lines:
        sys.exit(f"kernel {a.kernel} not found")
    meta = {}
    m = re.search(r"\.name:\s+(\S*" + re.escape(a.kernel) + r"\S*)", notes)
    if m:
        blk = notes[notes.rfind("- .", 0, m.start()):]
        for key in ("vgpr_count", "sgpr_count", "sgpr_spill_count", "vgpr_spill_count", "agpr_count",
                    "group_segment_fixed_size"):
            mm = re.search(r"\." + key + r":\s+(\d+)", blk)
            if mm:
                meta[key] = int(mm.group(1))
    res = {"kernel": a.kernel, "meta": meta, "instructions": len(lines), "loops": []}
    for n, (s, e) in enumerate(loops(lines)):
        h = collections.Counter(classify(mn, text) for _, mn, text in lines[s:e + 1])
        ent = {"loop": n, "offset": hex(lines[s][0]), "length": e - s + 1, "hist": dict(h.most_common())}
        valu = sum(v for k, v in h.items() if k.startswith("valu"))
        ent["valu"] = valu
        if a.rows:
            ent["per_row"] = {k: round(v / a.rows, 3) for k, v in h.items()}
            if a.levels:
                ent["valu_per_row_level"] = round(valu / (a.rows * a.levels), 3)
        res["loops"].append(ent)
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
