"""bench.py's rank launch (CPU, gloo): ``--gpus N`` without a torchrun environment must start N
ranks itself and the JSON line must report the world torch.distributed saw.  ``--dist-selftest``
runs the launch / shard / gather / timing machinery with a stand-in per-pair function on CPU
tensors (no model, no HIP), so this runs in the CPU suite."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 prints ONE line
    return json.loads(lines[0]), r.stderr


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    d, err = _run("--gpus", str(n), "--dist-selftest", "--steps", "2", "--warmup", "1")
    assert "launching %d ranks" % n in err
    assert d["n_gpus"] == n and d["world_size"] == n
    assert d["backend"] == "gloo"
    assert d["gathered_ok"] is True
    assert "not a measurement" in d["data"]
    # a multi-rank line carries parity of pair 0 (rank 0's) and of the last pair (the last rank's,
    # through the all-gather) -- the model bench builds the same block from the CPU oracle
    B = 2 * n
    assert d["parity"]["pairs_checked"] == [0, B - 1]
    assert d["parity"]["max_abs_dd_px"] == 0.0 and d["parity"]["ok"] is True
    # the attribution a multi-GPU line carries: every rank's step time and phase split, the world
    # size each rank's process group reported
    assert d["ranks"] == list(range(n)) and d["rank_world_size"] == [n] * n
    for k in ("per_rank_ms", "scatter_ms", "run_ms", "allgather_ms"):
        assert len(d[k]) == n and all(v >= 0.0 for v in d[k]), (k, d[k])
    assert all(s + r + g <= p * 1.5 + 1.0 for s, r, g, p in zip(d["scatter_ms"], d["run_ms"], d["allgather_ms"],
                                                                 d["per_rank_ms"]))


def test_gpus_1_single_process():
    d, err = _run("--gpus", "1", "--dist-selftest", "--steps", "2", "--warmup", "1")
    assert "launching" not in err
    assert d["n_gpus"] == 1 and d["world_size"] == 1
    assert d["parity"]["pairs_checked"] == [0]
