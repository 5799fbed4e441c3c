#!/usr/bin/env python3
"""Issue-cycle budget of a kernel's instruction stream, by pipe and instruction class.

    python tools/issue_budget.py LISTING.s KERNEL_SUBSTRING [--blocks B1,B2,...] [--per N]

LISTING.s is a hipcc -S listing (hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S ...).
Without --blocks the whole kernel body is counted once; with --blocks only those basic blocks
(e.g. the inner loop ".LBB0_118").  --per N divides the totals by N work units (e.g. the 512
(point, hidden) pairs one inner-loop iteration of bagproj_fwd covers per wave).

Costs are VALU-pipe cycles per wave64 instruction, measured on the MI355X by tools/valu_probe.hip
(independent chains, 3-4 waves per SIMD, normalised so that v_pk_fma_f32 = 4 cycles, the
fp32 VALU peak: 128 FMAs per 4 cycles per SIMD):

    v_pk_*                       4.0       (probe 5.39 raw)
    v_exp / v_rcp / v_log ...    6.7       (9.3 / 8.7 raw: about 1.7 x a packed FMA)
    v_bfi / v_bitop3 / v_perm    3.45      (4.65 raw)
    v_permlane*_swap             4.0       (assumed as a packed op)
    other VALU (v_fma, v_add...) 2.17      (2.92 raw: scalar fp32 runs at half the packed rate)
    v_mfma_f32_16x16x4_f32       32 matrix-pipe cycles, 8 of them holding the SIMD's vector
                                 issue (MI355X_MICROARCH.md constants table)
    v_mfma_f32_4x4x1_16b_f32     7.5 (probe: it does NOT overlap packed VALU)
    ds_* / s_nop                 counted; an s_nop N costs its wave N+1 issue slots

The VALU-pipe sum (VALU classes + MFMA issue holds) is the vector-issue bound of the stream on
one SIMD; the matrix pipe is a second bound; the larger of the two is the stream's floor.
"""
import re
import sys
from collections import Counter, OrderedDict

COST = OrderedDict([
    ("v_pk", 4.0), ("v_trans", 6.7), ("v_bitop", 3.45), ("v_permlane", 4.0), ("v_other", 2.17),
    ("mfma_issue", 8.0), ("s_nop", 4.0),
])
TRANS = ("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq", "v_sin", "v_cos")
MFMA_PIPE = {"v_mfma_f32_16x16x4_f32": 32.0, "v_mfma_f32_16x16x4f32": 32.0,
             "v_mfma_f32_4x4x1_16b_f32": 7.5, "v_mfma_f32_32x32x2_f32": 64.0}


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_pk_"):
        return "v_pk"
    if op.startswith(TRANS):
        return "v_trans"
    if op.startswith(("v_bfi", "v_bitop3", "v_perm_b32", "v_alignbit")):
        return "v_bitop"
    if op.startswith("v_permlane"):
        return "v_permlane"
    if op.startswith("v_"):
        return "v_other"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op == "s_nop":
        return "s_nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def kernel_blocks(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":")
                 or (l.startswith("_Z") and sym in l and ":" in l and not l.startswith("\t")))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name = OrderedDict(), [], "entry"
    for l in lines[start + 1:end]:
        s = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", s)
        if m:
            blocks[name] = cur
            name, cur = m.group(1), []
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur.append(s.split(";")[0].strip())
    blocks[name] = cur
    return blocks


def budget(instrs):
    cnt, cyc = Counter(), Counter()
    mfma_pipe = 0.0
    for s in instrs:
        op = s.split()[0]
        c = classify(op)
        cnt[c] += 1
        if c == "mfma":
            base = op.replace("_e64", "")
            mfma_pipe += MFMA_PIPE.get(base, 32.0)
            cyc["mfma_issue"] += COST["mfma_issue"]
        elif c == "s_nop":
            n = int(s.split()[1]) if len(s.split()) > 1 else 0
            cyc["s_nop"] += COST["s_nop"] * (n + 1)
        elif c in COST:
            cyc[c] += COST[c]
    return cnt, cyc, mfma_pipe


def main():
    args = sys.argv[1:]
    per, sel = 1.0, None
    if "--per" in args:
        i = args.index("--per")
        per = float(args[i + 1])
        del args[i:i + 2]
    if "--blocks" in args:
        i = args.index("--blocks")
        sel = args[i + 1].split(",")
        del args[i:i + 2]
    blocks = kernel_blocks(args[0], args[1])
    instrs = [s for b, ins in blocks.items() if sel is None or b in sel for s in ins]
    cnt, cyc, mpipe = budget(instrs)
    vec = sum(cyc.values())
    print(f"instructions: {len(instrs)}  " + " ".join(f"{k}={v}" for k, v in sorted(cnt.items())))
    print(f"{'class':12s} {'count':>7s} {'cycles':>9s} {'share':>7s}" + (f" {'per unit':>9s}" if per != 1 else ""))
    for k in COST:
        if cyc[k]:
            n = cnt["mfma"] if k == "mfma_issue" else cnt[k]
            row = f"{k:12s} {n:7d} {cyc[k]:9.1f} {cyc[k] / vec:7.1%}"
            if per != 1:
                row += f" {cyc[k] / per:9.3f}"
            print(row)
    print(f"vector-issue pipe: {vec:.1f} cycles" + (f" ({vec / per:.3f} per unit)" if per != 1 else ""))
    print(f"matrix pipe:       {mpipe:.1f} cycles" + (f" ({mpipe / per:.3f} per unit)" if per != 1 else ""))
    print(f"floor (max):       {max(vec, mpipe):.1f} cycles, bound by the "
          f"{'vector-issue' if vec >= mpipe else 'matrix'} pipe")


if __name__ == "__main__":
    main()
