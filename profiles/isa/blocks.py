"""Basic blocks of one kernel (hipcc -S): per block VALU/trans/SALU/LDS/VMEM counts and its branch.

usage: python blocks.py <file.s> <kernel-symbol-substring> [first_ins last_ins]
"""
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from loopcount import classify, kernel_lines  # noqa: E402


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    hi = int(sys.argv[4]) if len(sys.argv) > 4 else 10 ** 9
    n, cur, cnt, first = 0, "entry", {}, 0
    def flush(term):
        if lo <= first <= hi and cnt:
            print(f"{cur:>12} [{first:5d}] " + " ".join(f"{k}={v}" for k, v in sorted(cnt.items())) + f"  -> {term}")
    for ln in kernel_lines(path, sub):
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            flush("fall")
            cur, cnt, first = m.group(1), {}, n
            continue
        if not s or s.startswith((";", ".")):
            continue
        s = s.split(";")[0].strip()
        if not s:
            continue
        for c in classify(s):
            cnt[c] = cnt.get(c, 0) + 1
        n += 1
        if re.match(r"^s_(cbranch_\w+|branch)\s", s):
            flush(s)
            cnt, first = {}, n
            cur = cur + "+"
    flush("end")


if __name__ == "__main__":
    main()
