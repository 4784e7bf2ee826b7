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
    w = workload("auto", 8)  # the n = 1 line's family: c2's shard per GPU (bench.py adds the c3full phase)
    assert (w["workload"], w["N"], w["Mt"], w.get("scaling")) == ("c2-weak", 10000, 400000, None)
    w = workload("c3full", 8)
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
    # the reference's own decompositions of the 2 cores: 1 x 2 in-process, 2 x 1 under mpiexec (MPICH), the
    # stated value the fastest of them (README.md:36-38, the per-marker OpenMP fork of src/data.cpp:356-361)
    lays = {(lay["np"], lay["omp"]): lay for lay in r["layouts"]}
    assert set(lays) == {(1, 2), (2, 1)}, r.get("layout_errors")
    assert r["value"] >= max(lay["it_per_s"] for lay in r["layouts"]) * (1 - 1e-4)
    assert (r["np"], r["omp"]) in lays and r["value_np1"] > 0


def test_stated_cpu_baseline_is_the_faster_measurement():
    sys.path.insert(0, ROOT)
    import bench

    port = {"value": 0.4, "unit": "VAMP iterations/s", "kind": "port", "cores": 16}
    ref = {"value": 0.9, "unit": "VAMP iterations/s", "kind": "reference", "cores": 16, "np": 16, "omp": 1,
           "sample": "s", "projected": True}
    line = bench.stated_cpu_baseline({"cpu_baseline": dict(port), "cpu_reference_ops": dict(ref)})
    assert line["cpu_baseline"]["kind"] == "reference" and line["cpu_baseline"]["value"] == 0.9
    assert line["cpu_port"] == port
    line = bench.stated_cpu_baseline({"cpu_baseline": dict(port), "cpu_reference_ops": dict(ref, value=0.1)})
    assert line["cpu_baseline"] == port and "cpu_port" not in line


def _lines(p):
    return [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_hung_rank_ends_in_one_failure_line():
    """A rank that stops answering (here: after the rendezvous, so rank 0
    waits in a barrier for it) ends the job at --deadline-s: rank 0's watchdog
    prints ONE JSON line with "error" and every rank's last stage, and the
    launcher exits non-zero, instead of the job hanging until the caller's
    own limit with nothing printed."""
    import time

    t0 = time.monotonic()
    p = _run("--gpus", "2", "--steps", "2", "--dry-run", "--dry-run-hang-rank", "1", "--deadline-s", "25")
    took = time.monotonic() - t0
    assert p.returncode != 0
    recs = _lines(p)
    assert len(recs) == 1, p.stdout
    rec = recs[0]
    assert rec["value"] is None and "deadline" in rec["error"] and rec["n_gpus"] == 2
    assert "hang" in rec["rank_stages"]["1"]["stage"] and rec["rank_stages"]["0"]["stage"] == "dry-run timed"
    assert took < 25 + 30, took


def test_hung_rank_under_torchrun():
    """The same under the driver's launcher (torchrun, WORLD_SIZE set): rank
    0's watchdog prints the line and exits; torchrun stops the hung rank."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--dry-run", "--dry-run-hang-rank", "1", "--deadline-s", "25"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert p.returncode != 0
    recs = _lines(p)
    assert len(recs) == 1, p.stdout + p.stderr[-3000:]
    assert "deadline" in recs[0]["error"] and "hang" in recs[0]["rank_stages"]["1"]["stage"]


class _Ranks:
    def __init__(self, world, rank=0):
        from types import SimpleNamespace as NS

        self.world, self.rank, self.local = world, rank, rank
        self.dist = NS(all_gather_object=lambda out, mine: out.__setitem__(slice(None), [mine] * len(out)))

    def max(self, v):
        return v

    def sum(self, v):
        return v * self.world

    def barrier(self):
        pass

    def bcast(self, obj):
        return obj

    def gather(self, obj):
        return [obj] * self.world


class _Wd:
    partial = None
    dir = "/nonexistent"
    t0 = 0.0

    def stage(self, what):
        self.cur = what


def _fake_window(calls):
    from types import SimpleNamespace as NS

    def fake(args, R, w, wd, steps, warmup, tag, keep=False):
        calls.append((tag, w["workload"], R.world, steps, warmup))
        per_pass_ms = 0.6 * w["N"] * w["Mt"] / 5e8 / R.world  # C2: 0.6 ms a pass
        z = NS(ms_total=0.0, ms_timed=0.0, timed=0, launches=0, bytes_total=0.0)
        op = NS(ms_total=8.3 * steps * per_pass_ms, ms_timed=10 * per_pass_ms, timed=10, launches=8.3 * steps,
                bytes_total=8.3 * steps * 8.0 * w["N"] * w["Mt"] / R.world)
        st = NS(ax=z, atx=z, op=op, coll=z, ax_k=[z] * 4, atx_k=[z] * 4, op_k=[op, z, z, z],
                a_passes_exec=8.3 * steps)
        el = steps * (8.3 * per_pass_ms + 0.3) * 1e-3
        res = {"el": el, "st": st, "summ": {"cg_iters": [7] * (steps + warmup), "ons_iters": [8] * (steps + warmup)},
               "ref_passes": 37.7, "setup": 0.1, "M": w["Mt"] // R.world, "nranks": R.world, "steps": steps,
               "warmup": warmup, "model": "linear", "beta": None, "opts": None, "barrier": None,
               "rank_times": [{"rank": r} for r in range(R.world)]}
        if keep:
            res["d"] = NS(kernel_name=lambda which, K, mode: "atax_team_kernel<2, 6, 2, 3, 2, true, 2>",
                          close=lambda: None, get_phen=lambda: None)
        return res

    return fake


def test_multi_rank_line_assembly(monkeypatch):
    """The n > 1 line's assembly (no GPU: the VAMP windows are stubbed): the
    value is c2-weak's, rank 0 measured the 1-GPU bases first, the configs[2]
    headline phase follows the main one, and the line is one JSON object with
    the bases it is read against."""
    sys.path.insert(0, ROOT)
    import bench
    from vampomi_amd.workloads import workload

    calls = []
    monkeypatch.setattr(bench, "vamp_window", _fake_window(calls))
    args = bench.parse_args(["--gpus", "4", "--steps", "20", "--warmup", "5"])
    line = bench.run_linear(args, _Ranks(4), _Wd(), workload("auto", 4), 0.0)
    json.dumps(line)
    assert [c[0] for c in calls] == ["basis same-problem", "basis c3big", "main", "headline"]
    assert calls[0][1:4] == ("c2-weak@1gpu", 1, 20) and calls[1][1:3] == ("c3big", 1)
    assert calls[2][1:3] == ("c2-weak", 4) and calls[3][1:4] == ("c3full", 4, 10)
    assert line["config"]["workload"] == "c2-weak" and line["scaling"] == "weak" and line["n_gpus"] == 4
    assert line["value"] == round(4 * 20 / ((8.3 * 0.6 + 0.3) * 20e-3), 4)
    sp = line["one_gpu"]["same_problem"]
    assert sp["n_gpus"] == 1 and sp["Mt"] == 200000 and 3.0 < sp["speedup_of_this_run"] < 4.0
    h = line["headline_c3full"]
    assert h["workload"] == "c3full" and h["Mt"] == 500000 and h["n_gpus"] == 4
    eq = h["one_gpu_equivalent"]
    assert eq["measured_in_this_job"] and 0.5 < eq["strong_scaling_efficiency"] < 1.2
    assert "n = 1 line" in line["scaling_basis"]

    # explicit c3full: the strong line itself carries the measured equivalent
    calls.clear()
    args = bench.parse_args(["--gpus", "2", "--steps", "20", "--warmup", "5", "--config", "c3full"])
    line = bench.run_linear(args, _Ranks(2), _Wd(), workload("c3full", 2), 0.0)
    assert [c[0] for c in calls] == ["basis c3big", "main"]
    assert line["scaling"] == "strong" and line["one_gpu_equivalent"]["measured_in_this_job"]


def _stub_library(monkeypatch):
    """The library's Python mirror (Data, Vamp) replaced by a stub: no GPU."""
    from types import SimpleNamespace as NS

    import vampomi_amd as va

    z = NS(ms_total=0.0, ms_timed=0.0, timed=0, launches=0, bytes_total=0.0)

    class Data:
        def __init__(self, N, Mt, rank=0, nranks=1, comm_id=None, device=-1):
            assert nranks == 1 or comm_id is not None
            self.N, self.Mt, self.M, self.nranks = N, Mt, Mt // nranks, nranks

        def generate(self, seed, kind):
            pass

        def simulate_phen(self, seed, lam, h2):
            return [0.0] * self.M

        simulate_phen_binary = simulate_phen

        def set_variant(self, w, v):
            pass

        def reset_stats(self):
            pass

        def set_timing(self, on, period=1):
            pass

        def sync(self):
            pass

        def stats(self):
            op = NS(ms_total=5.0, ms_timed=0.6, timed=1, launches=8, bytes_total=8 * 8.0 * self.N * self.M)
            return NS(ax=z, atx=z, op=op, coll=z, ax_k=[z] * 4, atx_k=[z] * 4, op_k=[op, z, z, z], a_passes_exec=8)

        def kernel_name(self, which, K, mode):
            return "k"

        def get_phen(self):
            return None

        def read_ceiling(self, reps=9):
            return {"us_med": 500.0, "bytes": 8.0 * self.N * self.M, "GBs": 8.0 * self.N * self.M / 500e-6 / 1e9,
                    "variant": "stub"}

        def close(self):
            pass

    class Vamp:
        def __init__(self, d, opts, true_signal=None):
            self.n = 0

        def begin(self):
            pass

        def step(self):
            self.n += 1

        @property
        def a_passes(self):
            return 37.7 * self.n, 8.3 * self.n

        def summary(self):
            return {"cg_iters": [7] * self.n, "ons_iters": [8] * self.n}

        def end(self):
            pass

    monkeypatch.setattr(va, "Data", Data)
    monkeypatch.setattr(va, "Vamp", Vamp)
    monkeypatch.setattr(va, "comm_unique_id", lambda: b"x" * va.UNIQUE_ID_BYTES)


def test_vamp_window_and_bases_with_a_stub_library(monkeypatch):
    """bench.py's real vamp_window / one_gpu_bases code over a stub of the
    library's Python mirror (no GPU): every leg of the n > 1 flow runs without
    a Python error, so the driver's first multi-GPU run cannot die on one."""
    sys.path.insert(0, ROOT)
    import bench
    from vampomi_amd.workloads import workload

    _stub_library(monkeypatch)
    args = bench.parse_args(["--gpus", "2", "--steps", "3", "--warmup", "1"])
    out = bench.one_gpu_bases(args, _Ranks(2), _Wd(), workload("auto", 2), True)
    assert set(out) == {"same_problem", "c3big"}, out
    assert "error" not in out["same_problem"] and "error" not in out["c3big"], out
    line = bench.run_linear(args, _Ranks(2), _Wd(), workload("auto", 2), 0.0)
    json.dumps(line)
    assert "error" not in line["headline_c3full"], line["headline_c3full"]


def test_rehearsal_flow_with_a_stub_library(monkeypatch, capsys):
    """bench.py --rehearse P (the n > 1 flow with P loopback rank threads on one
    GPU, tests/test_gpu_bench.py runs it on the device) over the stub library:
    one line, rank 0's bases, the main phase and the headline phase at the
    scaled marker counts, per-rank records gathered from every thread."""
    sys.path.insert(0, ROOT)
    import bench

    _stub_library(monkeypatch)
    monkeypatch.setenv("TMPDIR", os.environ.get("TMPDIR", "/tmp"))
    args = bench.parse_args(["--rehearse", "3", "--rehearse-scale", "0.1", "--steps", "2", "--warmup", "1",
                             "--deadline-s", "120"])
    try:
        rc = bench.rehearse(args)
    finally:
        bench.WORKLOAD_SCALE = 1.0
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert rc == 0 and line["rehearsal"]["errors"] == [], line
    assert line["n_gpus"] == 3 and line["config"]["workload"] == "c2-weak" and line["config"]["Mt"] == 15000
    assert [r["rank"] for r in line["per_rank"]] == [0, 1, 2]
    assert "error" not in line["one_gpu"]["same_problem"] and "error" not in line["one_gpu"]["c3big"]
    h = line["headline_c3full"]
    assert "error" not in h and h["Mt"] == 50000 and h["n_gpus"] == 3


def test_same_run_ceiling_fields():
    """The n = 1 line's roofline carries the read ceiling measured on the same
    device after the timed region, and its fraction; not at n > 1, not with
    --no-read-ceiling, and a failing measurement never fails the line."""
    from types import SimpleNamespace as NS

    sys.path.insert(0, ROOT)
    import bench

    class D:
        def read_ceiling(self, reps):
            return {"us_med": 571.4, "bytes": 4.0e9, "GBs": 7000.0, "variant": "v"}

    class Bad:
        def read_ceiling(self, reps):
            raise RuntimeError("no")

    roof = {"achieved": 6500.0}
    bench.same_run_ceiling(NS(no_read_ceiling=False), D(), roof, 1)
    assert roof["frac_of_read_ceiling_same_run"] == round(6500.0 / 7000.0, 4)
    assert roof["read_ceiling_same_run"]["GBs"] == 7000.0
    for args, n in ((NS(no_read_ceiling=False), 2), (NS(no_read_ceiling=True), 1)):
        r = {"achieved": 1.0}
        bench.same_run_ceiling(args, D(), r, n)
        assert "read_ceiling_same_run" not in r
    r = {"achieved": 1.0}
    bench.same_run_ceiling(NS(no_read_ceiling=False), Bad(), r, 1)
    assert "error" in r["read_ceiling_same_run"] and "frac_of_read_ceiling_same_run" not in r
    bench.same_run_ceiling(NS(no_read_ceiling=False), D(), None, 1)  # no roofline: nothing to do
