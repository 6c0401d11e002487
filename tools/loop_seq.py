"""Instruction-class sequence of the MFMA-heaviest basic block of a kernel in a hipcc
--save-temps .s file (M mfma, V valu, L lds, W s_waitcnt, B barrier, S salu, G vmem),
plus its s_waitcnt list: shows whether operand reads run ahead of the MFMAs."""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    out, on = [], False
    for l in open(path):
        l = l.rstrip("\n")
        if not on and re.match(r"^_Z\S*%s\S*:" % re.escape(pat), l):
            on = True
            continue
        if on and l.startswith(".Lfunc_end"):
            break
        if on:
            out.append(l)
    labs = [i for i, l in enumerate(out) if re.match(r"^\.LBB", l)] + [len(out)]
    best = max(zip(labs, labs[1:]), key=lambda ab: sum("mfma" in l for l in out[ab[0]:ab[1]]))
    seq, waits = [], []
    for l in out[best[0]:best[1]]:
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")):
            continue
        op = t[0]
        seq.append("M" if "mfma" in op else "V" if op.startswith("v_") else "L" if op.startswith("ds_") else
                   "W" if op.startswith("s_waitcnt") else "B" if "barrier" in op else "S" if op.startswith("s_")
                   else "G")
        if op.startswith("s_waitcnt"):
            waits.append(" ".join(t[1:]))
    print("".join(seq))
    print(waits)


if __name__ == "__main__":
    main()
