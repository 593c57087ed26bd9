"""CPU: ``python bench.py --gpus N`` launches its own N ranks (torch.distributed.run child process)
when no launcher environment is present, and refuses loudly when fewer GPUs are visible.

The rank processes run ``--selftest-cpu``: gloo + the torch stand-in kernels of
tests/cpu_kernels.py on a 400-node graph (the launcher / sharding path, not a measurement)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_gpus2_self_launches_two_ranks():
    rc, res, err = _run("--gpus", "2", "--selftest-cpu", "--steps", "2", "--warmup", "1")
    assert rc == 0, err[-3000:]
    assert res["n_gpus"] == 2 and res["steps"] == 2
    assert res["config"]["parallelism"].startswith("dst-row shard x2")
    rows, nnz = res["shard"]["rows_per_rank"], res["shard"]["nnz_per_rank"]
    assert sum(rows) == 400 and abs(nnz[0] - nnz[1]) <= 0.02 * sum(nnz)
    assert res["value"] > 0 and res["final_loss"] == res["final_loss"]
    # every collective of the step timed in the eager pass, with its modeled time beside it
    col = res["collectives"]
    assert col["world_size"] == 2 and col["process_group_size"] == 2 and col["ranks_counted_by_all_reduce"] == 2
    assert col["backend"] == "gloo"
    # the "auto" form at 2 ranks is xagg: the flat gradient beside the edge pass, then g (slab form:
    # the gradient in two buckets)
    names = {"coords_all_gather", "loss_all_reduce", "grad_all_reduce", "g_all_reduce"}
    assert names <= set(col["measured_us"]), col["measured_us"].keys()
    for k, v in col["measured_us"].items():
        assert v["calls"] == 2 and v["avg_us"] > 0 and v["min_us"] <= v["avg_us"], (k, v)
        assert v["kind"] in ("all_gather", "all_reduce") and v["bytes"] > 0, (k, v)
        assert col["modeled_us"][k] > 0, k


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") not in (None, ""), reason="GPU box")
def test_bench_gpus_more_than_visible_fails_loudly():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    rc, res, err = _run("--gpus", str(n), "--steps", "1", "--warmup", "1", timeout=120)
    assert rc != 0
    assert res is not None and "error" in res
