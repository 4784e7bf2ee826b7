"""bench.py — VAMP iterations/s + HBM GB/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config auto|c2|c3full|c3|c3big|c4|c4full|c5]
                    [--no-cpu-baseline]

A "step" is one VAMP iteration (src/vamp.cpp:148-428) of the linear model
(or src/vamp_probit.cpp:68-463 of the probit model for c4) over the whole
synthetic problem, with every vector and the fp64 design matrix already
resident in HBM.  --stop-criteria-thr is 0, so exactly W+K iterations run; W
are untimed.

Workloads (synthetic, generated on the device):
  auto (default)  n = 1: c2; n > 1: c3full (the metric's own problem).
  c2      N=10,000 x Mt=50,000 i.i.d. Gaussian design (BASELINE configs[1]);
          with n > 1: weak scaling over markers (the reference's own
          sharding): N = 10,000, Mt = 50,000*n, 4 GB per GPU ("c2-weak").
  c3full  N=100,000 x Mt=500,000 methylation-like (configs[2], 400 GB) fixed,
          markers sharded over n >= 2 GPUs (strong scaling; 200 GB per GPU at
          n = 2, 50 GB at n = 8); value = iterations/s of the whole problem.
  c3      per-GPU shard of configs[2] (N=100,000 x 62,500 markers per GPU);
          weak; at n=8 it is exactly configs[2].
  c3big   N=100,000 x 300,000 markers per GPU (240 GB resident on one GPU).
  c4      probit model (configs[3]): N=50,000 x 50,000 markers per GPU; n=4
          is exactly configs[3].  c4full: configs[3] whole (80 GB) on any n.
  c5      LOO association test (configs[4]): N=100,000 x 62,500 markers per
          GPU; n=8 is exactly configs[4]; value = markers tested per second.

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) this process
is one rank; with `--gpus N` and no WORLD_SIZE it starts N rank processes
itself (127.0.0.1 rendezvous) before touching the GPU and exits with their
status; rank 0 prints the line.  The data path uses libvampomi's RCCL
communicator; torch.distributed (gloo) only broadcasts its id, runs the
barriers and takes the max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PMC_FILES = [os.path.join(ROOT, "profiles", f)
             for f in ("r03z_pmc_traffic_{}.json", "r03y_pmc_traffic_{}.json", "r03l_pmc_traffic_{}.json",
                       "r03g_pmc_traffic_{}.json",
                       "r03f_pmc_traffic_{}.json", "r03e_pmc_traffic_{}.json", "r02j_pmc_traffic_{}.json",
                       "r02i_pmc_traffic_{}.json", "r02h_pmc_traffic_{}.json", "r02_pmc_traffic_{}.json",
                       "r01_pmc_traffic_{}.json")]


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="auto", choices=["auto", "c2", "c3full", "c3", "c3big", "c4", "c4full", "c5"])
    ap.add_argument("--seed", type=int, default=20250711)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=45.0, help="seconds of host time for the CPU baseline")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event kernel timing")
    ap.add_argument("--timing-period", type=int, default=4,
                    help="time one A/A^T launch in this many of each (kernel, K) with HIP events (positions chosen "
                         "by a hash of the launch index; every launch timed costs 1-2.6 %% of a C2 iteration, "
                         "profiles/r03t_event_fence_ab.txt)")
    ap.add_argument("--batch-rhs", type=int, default=4)
    ap.add_argument("--op-variant", type=int, default=None,
                    help="one-pass operator plan (development hook, vampomi_dev_set_variant(ctx, 3, v))")
    ap.add_argument("--write", nargs="?", const=os.environ.get("TMPDIR", "/tmp"), default=None, metavar="DIR",
                    help="also time the same window with the per-iteration output files on (the main_meth.exe "
                         "drop-in rate: _it_K.bin, _r1_it_K.bin and CSV rows into a fresh directory under DIR)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rendezvous / max-over-ranks path only: no GPU work (CPU tests)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher: `python bench.py --gpus N` outside torchrun
# ---------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """Start n rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set; one GPU each).  Runs before this process imports torch or
    touches the GPU.  Rank 0 prints the JSON line on the shared stdout.  If a
    rank fails, the others are stopped; returns the first failing rank's code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VAMPOMI_RUN_ID=f"bench-{os.getpid()}-{port}")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # a rank failed: do not leave the others waiting in a collective
                    q.kill()
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------------------
# measurement helpers
# ---------------------------------------------------------------------------
def pmc_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` on `workload` from the committed
    rocprofv3 --pmc summary (tools/pmc.sh: FETCH_SIZE x2 gfx950 correction +
    WRITE_SIZE), newest round first; (bytes, file) or (None, None)."""
    for pat in PMC_FILES:
        f = pat.format(workload)
        try:
            base = kernel[:-1] if kernel.endswith(">") else kernel  # the profile's name may carry more
            for name, d in json.load(open(f)).items():                # template arguments after these
                at = name.find(base)
                if at >= 0 and name[at + len(base):at + len(base) + 1] in (">", ","):
                    return d.get("traffic_bytes_per_launch"), os.path.relpath(f, ROOT)
        except Exception:
            continue
    return None, None


def roofline(ks, kname: str, workload: str, period: int) -> dict:
    """The dominant kernel's achieved GB/s: algorithmic bytes per launch (exact
    count) over its average launch time (HIP events recorded in
    the dispatch packets of the sampled launches, on the stream they run on)."""
    avg_ms = ks.ms_timed / ks.timed
    bytes_per = ks.bytes_total / ks.launches
    achieved = bytes_per / (avg_ms * 1e-3) / 1e9
    traffic, tfile = pmc_traffic(kname, workload)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": int(traffic) if traffic else None,
            "traffic_unit": f"HBM bytes per launch (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, {tfile})"
            if tfile else None,
            "algorithmic_bytes_per_launch": int(bytes_per), "kernel": kname,
            "avg_launch_us": round(avg_ms * 1e3, 2), "launches": int(ks.launches), "timed_launches": int(ks.timed),
            "timing": f"HIP events in the dispatch packets of 1 in {max(1, period)} launches of each (kernel, K) "
                      "over the timed region (positions hashed from the launch index); launch counts exact"}


def cpu_baseline(d, w: dict, beta, seed: int, warmup: int, steps: int, gpu_ref_passes: float,
                 budget_s: float) -> dict:
    """The CPU oracle (C restatement, OpenMP) on the same workload.  Where
    W + k iterations fit the budget, it times the GPU's own window, iterations
    W+1..W+k (k <= K); otherwise it times iterations 1-2 per
    reference-equivalent A-pass and projects the GPU window's pass count."""
    import numpy as np  # noqa: F401
    from oracle import pyoracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    N, Mt, model = w["N"], w["Mt"], w.get("model", "linear")
    t0 = time.perf_counter()
    X = O.generate_markers(seed, w["kind"], N, 0, Mt)  # bit-identical to the device shard
    tgen = time.perf_counter() - t0
    y = d.get_phen()
    probe = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=2, stop_criteria_thr=0.0, keep_hist=False, model=model)
    t_it = probe["it_end_s"][-1] / 2
    k = max(0, min(steps, int((budget_s - warmup * t_it) / max(t_it, 1e-3))))
    base = {"unit": "VAMP iterations/s", "cores": threads, "kind": "port"}
    if k >= 2:
        r = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=warmup + k, stop_criteria_thr=0.0, keep_hist=False,
                          model=model)
        end = r["it_end_s"]
        win = end[warmup + k - 1] - (end[warmup - 1] if warmup > 0 else 0.0)
        return dict(base, value=k / win,
                    sample=f"iterations {warmup + 1}-{warmup + k} of {w['workload']} (N={N}, Mt={Mt}), the GPU "
                           f"window's first {k}, on {threads} OpenMP threads; data generation ({tgen:.1f} s) and "
                           f"iterations 1-{warmup} not timed",
                    cg_iters=[int(a) for a in r["cg_iters"][warmup:]], ons_iters=[int(a) for a in r["ons_iters"][warmup:]])
    per_pass = probe["it_end_s"][-1] / max(int(probe["a_passes"]), 1)
    return dict(base, value=1.0 / (per_pass * gpu_ref_passes), projected=True,
                sample=f"iterations 1-2 of {w['workload']} (N={N}, Mt={Mt}) on {threads} OpenMP threads: "
                       f"{per_pass * 1e3:.1f} ms per reference-equivalent A-pass, times the GPU window's "
                       f"{gpu_ref_passes:.2f} passes per iteration (W + k iterations exceed the {budget_s:.0f} s budget)")


def cpu_reference_ops(w: dict, seed: int, threads: int, k_cg: float):
    """The reference's OWN Ax / ATx (src/data.cpp:294-373, compiled from its
    sources into oracle/_ref/ref_data in the build container) timed on a
    generated matrix of the workload's shape, on the same host threads; the
    projected reference iteration rate uses its own call counts per
    iteration (it > 1): 5 + k Ax and 3 + k ATx with k = k1 + k2 CG steps
    (src/vamp.cpp:232,303,508,518-519,653-654,681,826), k from
    the GPU window.  The denoiser/EM (< 1 % of its CPU time) is left out."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_data")
    if not os.path.exists(exe):
        return {"skipped": "oracle/_ref/ref_data not built (needs /root/reference in the build container)"}
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.run([exe, "time", str(w["N"]), str(w["Mt"]), "2", str(seed)], env=env, capture_output=True,
                         text=True, timeout=300)
    if out.returncode != 0:
        return {"error": f"ref_data exit {out.returncode}: {out.stderr[-300:]}"}
    r = json.loads(out.stdout.strip().splitlines()[-1])
    t_it = ((5 + k_cg) * r["ax_ms"] + (3 + k_cg) * r["atx_ms"]) * 1e-3
    return {"value": 1.0 / t_it, "unit": "VAMP iterations/s", "kind": "reference", "projected": True,
            "cores": r["threads"], "ax_ms": r["ax_ms"], "atx_ms": r["atx_ms"],
            "sample": f"Ax and ATx (mean of 2 calls each) of the reference's src/data.cpp (oracle/_ref) on a generated "
                      f"{w['N']} x {w['Mt']} matrix, {r['threads']} OpenMP threads; iteration = (5 + k) Ax + (3 + k) "
                      f"ATx, k = {k_cg:.2f} (the GPU window's mean CG + Onsager steps)"}


def write_rate(args, d, R, opts, beta, barrier, el_nowrite: float) -> dict:
    """The same W + K iterations again with the reference's per-iteration
    output on (src/vamp.cpp:235-249 _it_K.bin / _r1_it_K.bin, :388-393 CSV
    rows) into a fresh directory under args.write: what a main_meth.exe user
    gets per iteration, with the main window's kernel timing, so the two
    windows differ only by the writes."""
    import dataclasses
    import shutil
    import tempfile

    import vampomi_amd as va

    out = tempfile.mkdtemp(prefix="vampomi_bench_", dir=args.write) if R.rank == 0 else None
    if R.world > 1:
        obj = [out]
        R.dist.broadcast_object_list(obj, src=0)
        out = obj[0]
    try:
        d.set_timing(not args.no_timing, args.timing_period)  # as in the main window: the ratio is the writes'
        v = va.Vamp(d, dataclasses.replace(opts, out_dir=out, out_name="bench"), true_signal=beta)
        v.begin()
        for _ in range(args.warmup):
            v.step()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            v.step()
        barrier()
        el = R.max(time.perf_counter() - t0)
        v.end()
        files = sorted(os.listdir(out))
        nbytes = sum(os.path.getsize(os.path.join(out, f)) for f in files)
    finally:
        R.barrier()
        if R.rank == 0:
            shutil.rmtree(out, ignore_errors=True)
    return {"elapsed_s": el, "ms_per_step": round(el / args.steps * 1e3, 3),
            "rate_vs_no_write": round(el_nowrite / el, 4), "files": len(files), "bytes_written": int(nbytes),
            "out_dir": args.write,
            "what": "the same iterations with _it_K.bin, _r1_it_K.bin (every iteration, every rank) and the CSV rows "
                    "written (async writer thread, writer.h); HIP-event timing as in the main window"}


def per_rank_times(R, st, el: float) -> list:
    """Per-rank device time of the A-kernels / the one-pass operator and the
    wall time of the window, gathered on rank 0 (a multi-GPU run's straggler
    shows up here)."""
    mine = {"rank": R.rank, "wall_s": round(el, 4),
            "op_ms_avg": round(st.op.ms_timed / st.op.timed, 4) if st.op.timed else None,
            "op_launches": int(st.op.launches),
            "a_kernels_ms": round(st.ax.ms_total + st.atx.ms_total + st.op.ms_total, 3),
            # RCCL all-reduces: HIP events on the stream around each (the wait
            # for the slowest rank included), count and bytes
            "allreduce_launches": int(st.coll.launches),
            "allreduce_ms_total": round(st.coll.ms_total, 3),
            "allreduce_us_avg": round(st.coll.ms_timed / st.coll.timed * 1e3, 2) if st.coll.timed else None,
            "allreduce_bytes": int(st.coll.bytes_total)}
    if R.world == 1:
        return [mine]
    out = [None] * R.world
    R.dist.all_gather_object(out, mine)
    return out


def cpu_baseline_assoc(d, w: dict, est, seed: int) -> dict:
    """The oracle's LOO test (OpenMP) on the first Ms markers of the same workload."""
    from oracle import pyoracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    N = w["N"]
    Ms = 8000
    X = O.generate_markers(seed, w["kind"], N, 0, Ms)
    y = d.get_phen()
    t0 = time.perf_counter()
    O.assoc_loo(X, y, est[:Ms])
    el = time.perf_counter() - t0
    return {"value": Ms / el, "unit": "markers/s", "cores": threads, "kind": "port",
            "sample": f"LOO test of markers 0-{Ms - 1} of {w['workload']} (N={N}, A.x over those markers) on "
                      f"{threads} OpenMP threads, {el:.1f} s"}


# ---------------------------------------------------------------------------
# the runs
# ---------------------------------------------------------------------------
class Ranks:
    """torch.distributed (gloo) for the id broadcast, barriers and max-over-ranks time."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        import torch.distributed as dist

        self.dist = dist
        if self.world > 1:
            dist.init_process_group("gloo")

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch

        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch

        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t)
        return float(t.item())

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def dry_run(args, R: Ranks):
    """The launcher, rendezvous, barrier and max-over-ranks path without a GPU."""
    R.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    R.barrier()
    el = R.max(time.perf_counter() - t0)
    seen = int(R.sum(1.0))
    if R.rank == 0:
        print(json.dumps({"metric": "dry run", "value": 0.0, "unit": "none", "n_gpus": R.world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
                          "ranks_seen": seen, "dry_run": True}), flush=True)
    R.close()


def bench_assoc(args, d, w, R: Ranks, t_start):
    """--config c5: the LOO association test (src/main_meth.cpp:245-264) on
    device-resident inputs; a step is one whole test."""
    import ctypes as C

    import numpy as np
    import torch

    import vampomi_amd as va

    N, Mt = w["N"], w["Mt"]
    beta = d.simulate_phen(args.seed + 1, lam=0.1, h2=0.5)
    t_setup = time.perf_counter() - t_start
    est = beta * 0.9 / np.sqrt(N)  # an estimate file's values (x1_hat / sqrt(N))
    dev = torch.device("cuda", R.local)
    e_t = torch.from_numpy(est).to(dev)
    p_t = torch.zeros(max(d.M, 1), dtype=torch.float64, device=dev)
    lib = va.load()

    def step():
        va._lib.check(lib.vampomi_assoc_loo(d.ctx, C.c_void_p(e_t.data_ptr()), C.c_void_p(p_t.data_ptr()), None,
                                            va.MEM_DEVICE))

    for _ in range(args.warmup):
        step()
    d.reset_stats()
    d.set_timing(not args.no_timing, args.timing_period)

    def barrier():
        d.sync()
        torch.cuda.synchronize()
        R.barrier()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    el = R.max(time.perf_counter() - t0)
    st = d.stats()
    roof = None
    if st.loo.timed:
        roof = roofline(st.loo, d.kernel_name(2, 1, 0), w["workload"], args.timing_period)
        roof["ax_avg_launch_us"] = round(st.ax.ms_timed / max(st.ax.timed, 1) * 1e3, 2)
    line = {
        "metric": "LOO association test: markers tested/s (+ achieved HBM GB/s of the per-marker pass)",
        "value": round(Mt * args.steps / el, 1),
        "unit": "markers/s",
        "n_gpus": R.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (index-keyed dyadic generator, generated in HBM)",
        "config": {"workload": w["workload"], "model": "association_test loo", "N": N, "Mt": Mt, "M_per_gpu": d.M,
                   "design": "methylation-like", "parallelism": f"markers sharded over {R.world} GPU(s)"},
        "roofline": roof,
        "setup_s": round(t_setup, 2),
        "cpu_baseline": None,
    }
    if R.rank == 0 and R.world == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline_assoc(d, w, est, args.seed)
        except Exception as e:
            line["cpu_baseline"] = {"error": repr(e)}
    d.close()
    if R.rank == 0:
        print(json.dumps(line), flush=True)
    R.close()


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # start the ranks before this process touches the GPU (or imports torch)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    import torch  # noqa: F401  (before libvampomi: one HIP runtime per process)

    R = Ranks()
    if args.dry_run:
        return dry_run(args, R)
    if args.gpus != R.world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={R.world}: launch one process per GPU")

    import vampomi_amd as va
    from vampomi_amd.workloads import workload

    if torch.cuda.is_available():
        torch.cuda.set_device(R.local)  # torch's own context on this rank's GPU, not on GPU 0
    n = R.world
    w = workload(args.config, n)
    N, Mt = w["N"], w["Mt"]
    comm_id = None
    if n > 1:
        obj = [va.comm_unique_id() if R.rank == 0 else None]
        R.dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    d = va.Data(N, Mt, rank=R.rank, nranks=n, comm_id=comm_id, device=R.local)
    t0 = time.perf_counter()
    d.generate(args.seed, w["kind"])
    model = w.get("model", "linear")
    if model == "loo":
        return bench_assoc(args, d, w, R, t0)
    if model == "bin_class":
        beta = d.simulate_phen_binary(args.seed + 1, lam=0.1, h2=0.8)
    else:
        beta = d.simulate_phen(args.seed + 1, lam=0.1, h2=0.8)
    t_setup = time.perf_counter() - t0
    if args.op_variant is not None:
        d.set_variant(3, args.op_variant)

    opts = va.VampOptions(max_iter=args.warmup + args.steps, stop_criteria_thr=0.0, batch_rhs=args.batch_rhs,
                          model=model)
    v = va.Vamp(d, opts, true_signal=beta)
    v.begin()
    for _ in range(args.warmup):
        v.step()
    ref0, _ = v.a_passes
    d.reset_stats()
    d.set_timing(not args.no_timing, args.timing_period)

    def barrier():
        d.sync()
        torch.cuda.synchronize() if torch.cuda.is_available() else None
        R.barrier()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        v.step()
    barrier()
    el = R.max(time.perf_counter() - t0)
    st = d.stats()
    rank_times = per_rank_times(R, st, el)
    ref1, _ = v.a_passes
    summ = v.summary()
    v.end()
    with_writes = write_rate(args, d, R, opts, beta, barrier, el) if args.write else None

    it_s = args.steps / el
    strong = w.get("scaling") == "strong"
    # dominant kernel: the (class, batch width) with the most device time
    cands = []
    for which, arr in ((0, st.ax_k), (1, st.atx_k), (3, st.op_k)):
        for k in range(4):
            if arr[k].timed:
                cands.append((arr[k].ms_total, which, k + 1, arr[k]))
    roof = None
    if cands:
        _, which, K, ks = max(cands, key=lambda c: c[0])
        # A^T.u in the CG carries the lmmse_mult epilogue (mode 1); the one-pass
        # operator's instantiation depends on N (passed as mode)
        roof = roofline(ks, d.kernel_name(which, K, N if which == 3 else 1), w["workload"], args.timing_period)
    all_ms = st.ax.ms_total + st.atx.ms_total + st.op.ms_total
    all_bytes = st.ax.bytes_total + st.atx.bytes_total + st.op.bytes_total
    ref_passes = (ref1 - ref0) / args.steps
    line = {
        "metric": "VAMP iterations/s (+ achieved HBM GB/s of the A/A^T kernels)",
        "value": round(it_s if strong else n * it_s, 4),
        "unit": "iterations/s" if (strong or n == 1) else "shard-iterations/s",
        "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (index-keyed dyadic generator, generated in HBM)",
        "config": {"workload": w["workload"], "model": model, "N": N, "Mt": Mt, "M_per_gpu": d.M,
                   "design": "gaussian" if w["kind"] == va.GEN_GAUSS else "methylation-like",
                   "iterations_timed": f"{args.warmup + 1}-{args.warmup + args.steps}",
                   "parallelism": f"markers sharded over {n} GPU(s)" + (", RCCL all-reduce" if n > 1 else ""),
                   "comm": {"backend": "rccl" if n > 1 else "none", "nranks": d.nranks}},
        "roofline": roof,
        "hbm_gbs_all_A_kernels": round(all_bytes / (all_ms * 1e-3) / 1e9, 1) if all_ms > 0 else None,
        "passes_exec_per_step": round(st.a_passes_exec / args.steps, 2),  # stats reset at the timed region
        "passes_ref_per_step": round(ref_passes, 2),
        # device time of the A-kernels over the wall time: each (kernel, K)'s
        # average over its sampled launches (hashed positions, unbiased over the
        # solve's steps) times its exact launch count; --timing-period 1 times
        # every launch (a measured sum, at 1-2.6 % of the iteration rate)
        "a_kernel_frac_of_step": round(all_ms * 1e-3 / el, 4) if el > 0 else None,
        "a_kernel_timing": {"timed_launches": int(st.ax.timed + st.atx.timed + st.op.timed),
                            "launches": int(st.ax.launches + st.atx.launches + st.op.launches),
                            "period": args.timing_period},
        "per_rank": rank_times,
        "cg_iters": summ["cg_iters"][args.warmup:], "ons_iters": summ["ons_iters"][args.warmup:],
        "setup_s": round(t_setup, 2),
        "cpu_baseline": None,
    }
    line["config"]["output_files"] = ("not written in the timed window (BASELINE.md: the metric excludes output-file "
                                      "writes); see with_writes" if args.write else
                                      "not written in the timed window (BASELINE.md: the metric excludes output-file "
                                      "writes; bench.py --write times them)")
    if with_writes:
        ws = with_writes.pop("elapsed_s")
        with_writes["value"] = round(args.steps / ws if strong else n * args.steps / ws, 4)
        line["with_writes"] = with_writes
    if strong and n > 1:
        # the problem does not fit one GPU.  ESTIMATE of its 1-GPU rate from the
        # committed c3big line (same N and design, 300,000 markers resident on
        # one MI355X, another run and build): its time per executed pass per
        # marker, times this run's markers and executed passes per iteration
        src = "profiles/r03e_bench_c3big.json"
        try:
            ref = json.load(open(os.path.join(ROOT, src)))
            per_pass_marker = ref["ms_per_step"] / (ref["passes_exec_per_step"] * ref["config"]["Mt"])
            one = 1e3 / (per_pass_marker * Mt * (st.a_passes_exec / args.steps))
            line["one_gpu_equivalent"] = {
                "estimate": True, "value": round(one, 4), "unit": "iterations/s",
                "source": f"{src} (N=100,000 x 300,000 on 1 GPU, {ref['ms_per_step']} ms per iteration at "
                          f"{ref['passes_exec_per_step']} passes): ms per pass per marker x Mt x this run's "
                          "passes per iteration; not a measurement of this problem on one GPU (it does not fit)",
                "strong_scaling_efficiency_estimate": round(it_s / (n * one), 4)}
        except Exception as e:
            line["one_gpu_equivalent"] = {"error": repr(e)}
    if model == "bin_class":
        line["parity_note"] = ("probit: x1_hat/r1 parity bar is max(1e-10, 10x the oracle's own rank-count spread), "
                               "integers exact (DESIGN.md §3)")
    if R.rank == 0 and n == 1 and not args.no_cpu_baseline and w["workload"] == "c3big":
        # the oracle's leg would generate the whole 240 GB matrix on the host
        line["cpu_baseline"] = {"skipped": "240 GB matrix; see the --config c3 line (same N, 62,500-marker shard)"}
    elif R.rank == 0 and n == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(d, w, beta, args.seed, args.warmup, args.steps, ref_passes,
                                                args.cpu_budget)
        except Exception as e:  # reported, never fatal for the GPU number
            line["cpu_baseline"] = {"error": repr(e)}
        if model == "linear":
            try:
                k_cg = (sum(line["cg_iters"]) + sum(line["ons_iters"])) / max(len(line["cg_iters"]), 1)
                threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
                line["cpu_reference_ops"] = cpu_reference_ops(w, args.seed, threads, k_cg)
            except Exception as e:
                line["cpu_reference_ops"] = {"error": repr(e)}
    d.close()
    if R.rank == 0:
        print(json.dumps(line), flush=True)
    R.close()


if __name__ == "__main__":
    main()
