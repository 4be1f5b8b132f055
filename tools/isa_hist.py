"""Static instruction histogram of one kernel in a hipcc -S assembly file.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
          --cuda-device-only -S csrc/preprocess.hip -o /tmp/pp.s
    python tools/isa_hist.py /tmp/pp.s med3_kernelILb1ELb1E [--blocks]

Counts are static (per instruction in the listing), so loop bodies count
once; --blocks prints the per-basic-block totals to find the hot body.
"""
import collections
import sys


def kernel_lines(path, needle):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if start is None and needle in l and l.split(";")[0].rstrip().endswith(":") \
                and not l.startswith("\t"):
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit(f"kernel matching {needle!r} not found")


def main():
    path, needle = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, needle)
    total = collections.Counter()
    blocks, cur, name = [], collections.Counter(), "entry"
    for l in body[1:]:
        s = l.split(";")[0].strip()
        if not s or s.startswith("."):
            if s.startswith(".LBB"):
                blocks.append((name, cur))
                cur, name = collections.Counter(), s.rstrip(":")
            continue
        op = s.split()[0]
        total[op] += 1
        cur[op] += 1
    blocks.append((name, cur))
    print("total", sum(total.values()))
    for k, v in total.most_common(50):
        print(f"{v:6d} {k}")
    if "--blocks" in sys.argv:
        for n, c in blocks:
            print(f"{n:12s} {sum(c.values()):6d}  " +
                  " ".join(f"{k}:{v}" for k, v in c.most_common(6)))


if __name__ == "__main__":
    main()
