"""Static instruction counts per basic block of one kernel in a gfx950 .s file.

Usage: python tools/asm_blocks.py FILE.s SYMBOL_SUBSTRING [--all]

Prints, per basic block (label), the number of VALU (v_*, MFMAs included as
SQ_INSTS_VALU counts them), MFMA, SALU, DS, VMEM (global/buffer) instructions
and the branch targets, so trip counts can be attached by hand.  Diagnostic
only (VALU attribution): never imported by the product.
"""
import re
import sys


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if l.endswith(":") and not l.startswith((".", "\t", " ")) and sub in l.split(":")[0] \
                or (sub in l and re.match(r"^_Z\S+:", l)):
            start = i
            break
    if start is None:
        raise SystemExit("symbol not found")
    end = start + 1
    while end < len(lines) and not lines[end].startswith(".Lfunc_end"):
        end += 1
    return lines[start:end]


def main():
    path, sub = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, sub)
    blocks = []
    cur = {"name": "entry", "v": 0, "mfma": 0, "s": 0, "ds": 0, "vm": 0, "br": [], "n": 0, "cats": {}}
    for l in body[1:]:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")):
            m = re.match(r"^(\.LBB\S+):", t)
            if m:
                blocks.append(cur)
                cur = {"name": m.group(1), "v": 0, "mfma": 0, "s": 0, "ds": 0, "vm": 0, "br": [], "n": 0,
                       "cats": {}}
            continue
        op = t.split()[0]
        cur["n"] += 1
        if op.startswith("v_"):
            cur["v"] += 1
            if "mfma" in op:
                cur["mfma"] += 1
            else:
                cur["cats"][op] = cur["cats"].get(op, 0) + 1
        elif op.startswith("s_"):
            cur["s"] += 1
            if op.startswith("s_cbranch") or op == "s_branch":
                cur["br"].append(t.split()[1])
        elif op.startswith("ds_"):
            cur["ds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            cur["vm"] += 1
    blocks.append(cur)
    tot = {"v": 0, "mfma": 0, "s": 0, "ds": 0, "vm": 0}
    for b in blocks:
        for k in tot:
            tot[k] += b[k]
        top = sorted(b["cats"].items(), key=lambda kv: -kv[1])[:6]
        print(f"{b['name']:>14}: valu {b['v']:5d} mfma {b['mfma']:4d} salu {b['s']:4d} ds {b['ds']:4d} "
              f"vmem {b['vm']:4d} -> {','.join(b['br'])}  {' '.join(f'{k}:{v}' for k, v in top) if '--all' in sys.argv else ''}")
    print("total", tot)


if __name__ == "__main__":
    main()
