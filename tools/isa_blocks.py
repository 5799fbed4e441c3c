#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (loop bodies marked).

    python tools/isa_blocks.py file.s SYMBOL_SUBSTRING
"""
import re
import sys
from collections import Counter


def main(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":") is False or (l.startswith("_Z") and sym in l and ":" in l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name = [], [], "entry"
    for l in lines[start + 1:end]:
        s = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            blocks.append((name, cur)); name, cur = s[:-1].split(":")[0], []
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur.append(s.split(";")[0].strip())
    blocks.append((name, cur))
    order = [b[0] for b in blocks]
    for bi, (nm, ins) in enumerate(blocks):
        c = Counter()
        loop = ""
        for s in ins:
            op = s.split()[0]
            if op.startswith("v_mfma"):
                c["mfma"] += 1
            elif op.startswith("v_pk_"):
                c["v_pk"] += 1
            elif op.startswith(("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq", "v_sin", "v_cos")):
                c["v_trans"] += 1
            elif op.startswith(("v_accvgpr",)):
                c["accvgpr"] += 1
            elif op.startswith("v_"):
                c["v_other"] += 1
            elif op.startswith("ds_"):
                c["ds"] += 1
            elif op.startswith(("global_", "buffer_")):
                c["vmem"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            if op.startswith("s_cbranch") or op == "s_branch":
                tgt = s.split()[-1]
                if tgt in order and order.index(tgt) <= bi:
                    loop += f" <-loop back to {tgt}"
        print(f"{nm:12s} n={len(ins):5d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())) + loop)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
