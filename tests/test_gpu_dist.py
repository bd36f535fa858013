"""Two ranks through the HIP path on one GPU (pytest -m gpu): bench.py --gpus 2 starts two rank
processes, each with its own wg_ctx on cuda:0 (--same-device) and the report's collectives over gloo
(--dist-backend gloo; RCCL refuses two ranks on one GPU). C3 is sharded by session (session s ->
rank s mod 2, dist.shard_packets); every rank seals and opens its 4M x 1420 B shard with k_step and
checks a seeded 2048-packet sample of its own ciphertext against the oracle, and a mismatch on any
rank fails the line. This is the multi-GPU code path the driver's 8-GPU run takes, minus RCCL
(exercised at world 1: profiles/r04_bench_c1_torchrun1.json). Reference: EstablishedSession.java:59-71
(disjoint sessions)."""
import json
import os
import subprocess
import sys

import pytest

from wgtest import ROOT

pytestmark = pytest.mark.gpu


def test_two_ranks_sharded_c3_on_one_gpu():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "c3",
                        "--steps", "2", "--warmup", "1", "--ramp-ms", "0", "--dist-backend", "gloo",
                        "--same-device"], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    j = json.loads(lines[-1])
    assert j["n_gpus"] == 2 and j["verified"] is True
    assert j["oracle_sample"]["bit_exact"] is True and j["oracle_sample"]["all_ranks_verified"] is True
    assert [r["rank"] for r in j["per_gpu"]] == [0, 1]
    assert sum(r["packets_per_step"] for r in j["per_gpu"]) == 8 * 1024 * 1024
    assert j["config"]["rehearsal"].startswith("2 ranks on cuda:0")
