"""bench.py's multi-GPU launch path on CPU: `python bench.py --gpus N` outside
torchrun starts N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_* on 127.0.0.1), they meet over gloo, and rank 0 prints the one line
with n_gpus = N.  --dry-run stops short of the GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    p = _run("--gpus", str(n), "--steps", "3", "--warmup", "1", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["ranks_seen"] == n and rec["steps"] == 3


def test_gpus_must_match_world_size():
    # under an external launcher (WORLD_SIZE set) --gpus must agree with it
    p = _run("--gpus", "2", "--steps", "1", env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)


def test_workload_selection():
    sys.path.insert(0, ROOT)
    from vampomi_amd.workloads import workload

    assert workload("auto", 1)["workload"] == "c2"
    w = workload("auto", 8)
    assert (w["workload"], w["N"], w["Mt"], w.get("scaling")) == ("c3full", 100000, 500000, "strong")
    assert workload("c3full", 2)["Mt"] == 500000
    with pytest.raises(ValueError):
        workload("c3full", 1)
    assert workload("c2", 4)["Mt"] == 200000 and workload("c3", 8)["Mt"] == 500000


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "ref_data")),
                    reason="oracle/_ref not built (needs /root/reference)")
def test_cpu_reference_ops_leg():
    """bench.py's kind-"reference" CPU leg: the reference's own Ax / ATx
    (src/data.cpp via oracle/_ref) timed on a small generated matrix, and the
    projection from its call counts per iteration."""
    sys.path.insert(0, ROOT)
    import bench

    r = bench.cpu_reference_ops({"N": 300, "Mt": 500, "workload": "tiny"}, 3, 2, 10.0)
    assert r["kind"] == "reference" and r["cores"] == 2 and r["ax_ms"] > 0 and r["atx_ms"] > 0
    want = 1.0 / ((15 * r["ax_ms"] + 13 * r["atx_ms"]) * 1e-3)
    assert abs(r["value"] - want) <= 1e-9 * want
