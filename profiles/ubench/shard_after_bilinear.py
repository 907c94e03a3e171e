"""Diagnostic (not part of the product): bench.shard_bench (group with the RCCL exchange, then the
plain step) with and without the bench's bilinear leg before it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
r = bench.shard_bench(torch, 0, "3d")
print("shard first:", r["sharded_ms_per_step"], r["plain_ms_per_step"], flush=True)
print("bilinear:", bench.bilinear_bench(torch, dev)["kernel_avg_ms"], flush=True)
r = bench.shard_bench(torch, 0, "3d")
print("shard after bilinear:", r["sharded_ms_per_step"], r["plain_ms_per_step"], flush=True)
r = bench.shard_bench(torch, 0, "3d")
print("shard again:", r["sharded_ms_per_step"], r["plain_ms_per_step"], flush=True)
