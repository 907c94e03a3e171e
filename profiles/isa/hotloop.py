"""Instruction mix of one loop's hot path (hipcc -S output), CPU-only analysis.

usage: python hotloop.py <file.s> <kernel-substring> <loop-header-label> [steps_per_iter]
Takes the blocks the compiler annotates as in that loop ("in Loop: Header=..." comments, the
header itself) and skips blocks that are cold by construction: spin-wait loops (s_sleep) and
IEEE redo / division fix-up blocks (v_div_scale).
"""
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from loopcount import kernel_lines  # noqa: E402


def main():
    path, sub, head = sys.argv[1], sys.argv[2], sys.argv[3]
    per = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    tag = head.lstrip(".").lstrip("L")
    blocks, cur, inloop = {}, None, set()
    for ln in kernel_lines(path, sub):
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):(.*)$", s)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            if cur == head or f"Header={tag} " in m.group(2) + " ":
                inloop.add(cur)
            continue
        if cur is None or not s or s.startswith((";", ".")):
            continue
        s = s.split(";")[0].strip()
        if s:
            blocks[cur].append(s)
    hot = {}
    for b in inloop:
        # basic blocks: split a labelled block after every branch
        sub, piece = [], []
        for x in blocks[b]:
            piece.append(x)
            if re.match(r"^s_(cbranch_\w+|branch)\b", x):
                sub.append(piece)
                piece = []
        if piece:
            sub.append(piece)
        for ins in sub:
            if any(x.startswith("s_sleep") for x in ins) or any(("v_div_scale" in x or "v_cmp_class" in x) for x in ins):
                continue
            for x in ins:
                op = x.split()[0]
                hot[op] = hot.get(op, 0) + 1
    tot = sum(hot.values())
    print(f"{head}: {tot} instructions on the hot path ({len(inloop)} blocks), {tot / per:.1f} per step")
    for k, v in sorted(hot.items(), key=lambda kv: -kv[1]):
        print(f"{v / per:7.1f} {k}")


if __name__ == "__main__":
    main()
