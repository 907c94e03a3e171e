"""Static instruction mix of a kernel's loops from hipcc -S output (CPU-only analysis).

usage: python loopcount.py <file.s> <kernel-symbol-substring> [min_valu]
Prints every backward-branch loop (label .. branch) with its VALU / transcendental /
packed / SALU / LDS / VMEM counts, counting each instruction of the range once.
"""
import re
import sys

TRANS = ("v_rcp_", "v_sqrt_", "v_rsq_", "v_exp_", "v_log_", "v_sin_", "v_cos_")


def kernel_lines(path, sub):
    out, on = [], False
    for ln in open(path):
        if not on and re.match(r"^_Z\S*" + re.escape(sub) + r"\S*:", ln):
            on = True
            continue
        if on:
            if ln.startswith(".Lfunc_end"):
                break
            out.append(ln.rstrip("\n"))
    return out


def classify(ins):
    m = ins.split()[0]
    if m.startswith("v_"):
        c = ["valu"]
        if m.startswith(TRANS):
            c.append("trans")
        if m.startswith("v_pk_"):
            c.append("pk")
        return c
    if m.startswith("s_waitcnt") or m.startswith("s_nop"):
        return ["wait"]
    if m.startswith("s_"):
        return ["salu"]
    if m.startswith("ds_"):
        return ["lds"]
    if m.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return ["vmem"]
    return ["other"]


def main():
    path, sub = sys.argv[1], sys.argv[2]
    minv = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lines = kernel_lines(path, sub)
    labels, ins = {}, []
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith((";", ".", "//")) and not re.match(r"^\.LBB\S+:", s):
            continue
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        s = s.split(";")[0].strip()
        if s:
            ins.append(s)
    tot = {}
    for i in ins:
        for c in classify(i):
            tot[c] = tot.get(c, 0) + 1
    print("kernel total:", tot, "instructions", len(ins))
    for j, i in enumerate(ins):
        m = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\S+)", i)
        if m and m.group(2) in labels and labels[m.group(2)] <= j:
            a = labels[m.group(2)]
            cnt = {}
            for k in ins[a:j + 1]:
                for c in classify(k):
                    cnt[c] = cnt.get(c, 0) + 1
            if cnt.get("valu", 0) >= minv:
                print(f"loop {m.group(2)} [{a}..{j}] len {j - a + 1}: {cnt}")


if __name__ == "__main__":
    main()
