"""CPU: `bench.py --gpus N` without an external launcher starts N rank
processes itself (torch.distributed.run, rendezvous on 127.0.0.1) and every
rank joins one process group.  Runs the bring-up alone (--launch-check) over
gloo, so no GPU is needed; the driver's 1->8 scaling run uses the same path
with RCCL."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bench_launches_n_ranks(n):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["UGPU_BENCH_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--launch-check"],
                         capture_output=True, timeout=240, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr.decode()[-2000:]
    lines = [l for l in out.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout.decode()
    j = json.loads(lines[0])
    assert j["n_gpus"] == n and j["backend"] == "gloo"
    assert sorted(r["rank"] for r in j["ranks"]) == list(range(n))
    assert sorted(r["local_rank"] for r in j["ranks"]) == list(range(n))
    assert len({r["pid"] for r in j["ranks"]}) == n  # one process per rank
    assert "launching %d ranks" % n in out.stderr.decode()
