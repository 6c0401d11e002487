"""Per-basic-block instruction mix of one kernel in a hipcc ``--save-temps`` .s file.

    python tools/asm_stats.py build.s 'gcn_fused_bwd2_kernelILi7ELi3ELi256ELi2ELi1E'

Prints, for every basic block of the first kernel whose symbol contains the pattern,
the counts of MFMA / VALU / SALU / LDS / VMEM instructions and the block's branch, so
that a loop body's VALU-per-MFMA ratio can be read before a GPU run."""
import collections
import re
import sys


def kernel_lines(path, pat):
    out, on = [], False
    for line in open(path):
        line = line.rstrip("\n")
        if not on and re.match(r"^_Z\S*%s\S*:" % re.escape(pat), line):
            on = True
            continue
        if on and line.startswith(".Lfunc_end"):
            break
        if on:
            out.append(line)
    return out


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return None


def main():
    path, pat = sys.argv[1], sys.argv[2]
    f = kernel_lines(path, pat)
    if not f:
        sys.exit("no kernel matching %r" % pat)
    labels = [i for i, l in enumerate(f) if re.match(r"^\.LBB\d+_\d+:", l)]
    starts = [0] + labels
    total = collections.Counter()
    for a, b in zip(starts, starts[1:] + [len(f)]):
        c = collections.Counter()
        for l in f[a:b]:
            t = l.strip().split()
            if not t or t[0].startswith((";", ".")):
                continue
            k = classify(t[0])
            if k:
                c[k] += 1
        total.update(c)
        br = [l.strip().split(";")[0] for l in f[a:b] if "s_cbranch" in l or "s_branch" in l]
        name = f[a].strip() if a in labels else "<entry>"
        print("%-14s %-60s %s" % (name, dict(c), br[-1] if br else ""))
    print("total", dict(total))


if __name__ == "__main__":
    main()
