"""Static instruction histogram of one kernel in a hipcc -S listing (gfx950): every mnemonic
between the kernel's label and its .Lfunc_end, VALU / packed-VALU / SALU / LDS totals.
usage: isa_ops.py LISTING.s KERNEL_LABEL_PREFIX [TOP]   (the first label starting with the prefix)"""
import collections
import re
import sys


def main():
    path, prefix = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and l.split(":")[0].endswith(("j", "E")) or
                 (l.startswith(prefix) and ":" in l and not l.startswith("\t")))
    ops = collections.Counter()
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        t = l.strip().split()
        if t and re.match(r"^[vsdgb][a-z_0-9]+$", t[0]):
            ops[t[0]] += 1
    tot = lambda pre: sum(c for o, c in ops.items() if o.startswith(pre))  # noqa: E731
    print("%s: VALU %d (packed %d), SALU %d, LDS %d, branches %d" % (
        lines[start].split(":")[0][:100], tot("v_"), tot("v_pk_"), tot("s_"), tot("ds_"), tot("s_cbranch")))
    for o, c in ops.most_common(top):
        print("  %-28s %d" % (o, c))


if __name__ == "__main__":
    main()
