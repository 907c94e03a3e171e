"""Static instruction count of the rollout chain's step (CPU-only; hipcc -S of the kernels).

usage: python profiles/isa/chain_count.py  -> writes profiles/isa/chain_count.json
The chain loop of mppi_rollout_roles_kernel<256, 3, 0, false> (two steps per iteration, the
verified-reciprocal cell path), counted by hotloop.py's rules (spin waits and the IEEE redo
blocks excluded).  bench.py reports it when src_sha256 matches the current kernel sources.
"""
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path[:0] = [HERE, ROOT]
import bench  # noqa: E402
from loopcount import kernel_lines  # noqa: E402

KERNEL = "roles_kernelILi256ELi3ELi0ELb0E"


def main():
    csrc = os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd", "csrc")
    out = os.path.join(tempfile.gettempdir(), "mppi_chain_count.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-slp-vectorize", f"-I{ROOT}/include", f"-I{csrc}", "-x", "hip", "--cuda-device-only", "-S",
                    os.path.join(csrc, "mppi_kernels.hip"), "-o", out], check=True, capture_output=True)
    # the chain loop: the first backward-branch loop with >= 100 packed instructions
    res = subprocess.run([sys.executable, os.path.join(HERE, "loopcount.py"), out, KERNEL], check=True,
                         capture_output=True, text=True).stdout
    head = next(m.group(1) for m in re.finditer(r"loop (\.LBB\S+) \[.*'pk': (\d+)", res) if int(m.group(2)) >= 100)
    hot = subprocess.run([sys.executable, os.path.join(HERE, "hotloop.py"), out, KERNEL, head, "2"], check=True,
                         capture_output=True, text=True).stdout
    per = float(re.search(r"([\d.]+) per step", hot).group(1))
    mix = {m.group(2): float(m.group(1)) for m in re.finditer(r"^\s+([\d.]+) (\S+)$", hot, re.M)}
    rec = {"src_sha256": bench.source_hash(), "kernel": "mppi_rollout_roles_kernel<256, 3, 0, false>",
           "loop": head, "instructions_per_step": per,
           "s_nop_per_step": mix.get("s_nop", 0.0), "frexp_per_step": mix.get("v_frexp_exp_i32_f32_e32", 0.0)}
    with open(os.path.join(HERE, "chain_count.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
    assert kernel_lines(out, KERNEL)


if __name__ == "__main__":
    main()
