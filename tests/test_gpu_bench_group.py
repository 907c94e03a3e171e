"""GPU: bench.py's in-process group path, the one `bench.py --gpus N` takes in one process (VERDICT r05
item 1): Runner(devices=...), mppi_group_create, member threads, solo_rate and the line's group fields.
Two members share device 0 (records exchanged by device copies); C2 size so it runs in seconds.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_group_line_fields():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c2", "--group-devices", "0,0",
           "--steps", "10", "--warmup", "2", "--prewarm-ms", "20", "--cpu-baseline-seconds", "0", "--no-c4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    c = d["config"]
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["steps"] == 10
    assert c["launcher"].startswith("one process, C-ABI group (mppi_group_create), member threads"), c["launcher"]
    assert "device-copy record exchange" in c["launcher"], c["launcher"]
    g = c["group"]
    assert g["members"] == 2 and g["devices"] == 1 and g["rccl"] == 0 and g["threaded"] == 1, g
    assert c["rccl_ranks"] == 0 and c["global_K"] == 4096 and c["k_per_gpu"] == 2048, c
    assert c["speedup_vs_1"] is not None and c["speedup_vs_1"] > 0
    # 8 leaves per member (a power of two): the group's controls equal one context's bit for bit
    assert c["group_parity_bitwise"] is True, c
    assert c["parallelism"].startswith("K-sharded over 2 members on 1 GPU(s)"), c["parallelism"]
