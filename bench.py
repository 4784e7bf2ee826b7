"""bench.py — VAMP iterations/s + HBM GB/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config auto|c2|c3full|c3|c3big|c4|c4full|c5]
                    [--no-cpu-baseline] [--no-read-ceiling] [--no-timing | --timing-period P]
                    [--rehearse P]   (the n > 1 flow with P loopback rank threads on one GPU)

The line's `roofline` is the dominant kernel's algorithmic bytes per launch
over its HIP-event launch time, against the 8 TB/s spec (`frac`), against the
pool's measured read ceiling (`frac_of_read_ceiling`, profiles/) and, at
n = 1, against a pure read stream of the same resident matrix measured by this
process right after the timed region (`frac_of_read_ceiling_same_run`).

A "step" is one VAMP iteration (src/vamp.cpp:148-428) of the linear model
(or src/vamp_probit.cpp:68-463 of the probit model for c4) over the whole
synthetic problem, with every vector and the fp64 design matrix already
resident in HBM.  --stop-criteria-thr is 0, so exactly W+K iterations run; W
are untimed.

Workloads (synthetic, generated on the device):
  auto (default)  c2 at every n: n = 1 is BASELINE configs[1]; n > 1 is its
          weak-scaling form c2-weak (50,000 markers per GPU), so the driver's
          1 -> 8 curve compares one workload family.  At n > 1 the same line
          also carries `headline_c3full`, configs[2] itself (N=100,000 x
          Mt=500,000, the metric's own problem) run in the same job, and the
          1-GPU bases both are read against, measured in the same job on
          rank 0's GPU before the n-rank phases (`one_gpu`).
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

Failure is bounded and reported: every rank runs a watchdog (--deadline-s,
default 420 s from the start) and records its stage (init / basis / generate
/ warmup / timed / cpu / ...) in a per-job directory under $TMPDIR; on expiry
rank 0 prints ONE JSON line with "error" and every rank's last stage and all
ranks exit non-zero (torchrun then stops the rest).  RCCL creation is
non-blocking and bounded (VAMPOMI_COMM_INIT_TIMEOUT_S, 90 s here) and a
collective that never completes fails after VAMPOMI_COLL_TIMEOUT_S (120 s
here), so a stuck transport ends in the same JSON line, not in silence.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time
import traceback

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PMC_FILES = [os.path.join(ROOT, "profiles", f)
             for f in ("r06zz_pmc_traffic_{}.json", "r06z_pmc_traffic_{}.json", "r05zz_pmc_traffic_{}.json", "r05z_pmc_traffic_{}.json", "r05_pmc_traffic_{}.json", "r04_pmc_traffic_{}.json", "r03z_pmc_traffic_{}.json", "r03y_pmc_traffic_{}.json", "r03l_pmc_traffic_{}.json",
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
    ap.add_argument("--no-read-ceiling", action="store_true",
                    help="skip the same-run HBM read ceiling (a pure read stream of the resident matrix, after the "
                         "timed region, n = 1)")
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
    ap.add_argument("--dry-run-hang-rank", type=int, default=-1,
                    help="(tests) with --dry-run: this rank stops answering after the rendezvous")
    ap.add_argument("--deadline-s", type=float, default=420.0,
                    help="the whole run's time limit: past it every rank stops and rank 0 prints a JSON line with "
                         "\"error\" and each rank's last stage (keep it under the caller's own limit)")
    ap.add_argument("--no-headline", action="store_true",
                    help="n > 1 with --config auto: skip the configs[2] (c3full) phase and its 1-GPU basis")
    ap.add_argument("--rehearse", type=int, default=0, metavar="P",
                    help="rehearsal of the n > 1 flow on ONE GPU: P loopback ranks as threads of this process on "
                         "GPU 0 (bases, main phase, headline phase, line assembly), every workload's markers "
                         "scaled by --rehearse-scale; the rate is not a multi-GPU number")
    ap.add_argument("--rehearse-scale", type=float, default=0.05)
    return ap.parse_args(argv)


WORKLOAD_SCALE = 1.0  # --rehearse: markers of every workload scaled by this


def get_workload(cfg: str, n: int) -> dict:
    from vampomi_amd.workloads import workload

    w = workload(cfg, n)
    if WORKLOAD_SCALE != 1.0:
        w = dict(w, Mt=max(n, int(round(w["Mt"] * WORKLOAD_SCALE))), rehearsal_scale=WORKLOAD_SCALE)
    return w


# ---------------------------------------------------------------------------
# launcher: `python bench.py --gpus N` outside torchrun
# ---------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, deadline_s: float) -> int:
    """Start n rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set; one GPU each).  Runs before this process imports torch or
    touches the GPU.  Rank 0 prints the JSON line on the shared stdout.  If a
    rank fails, the others are stopped; returns the first failing rank's code.
    The ranks' own watchdogs end the job at the deadline; if they cannot (a
    rank stuck where Python never runs again) this parent kills every rank
    a little later and prints the failure line itself, with the stages the
    ranks reported."""
    port = _free_port()
    run_id = f"bench-{os.getpid()}-{port}"
    t0 = time.time()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VAMPOMI_RUN_ID=run_id,
                   VAMPOMI_BENCH_T0=repr(t0))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else None, text=True))
    # relay rank 0's stdout, noting whether its JSON line came
    seen = {"line": False}

    def relay(f):
        for ln in f:
            if ln.startswith("{"):
                seen["line"] = True
            sys.stdout.write(ln)
            sys.stdout.flush()

    th = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    th.start()
    rc = 0
    live = list(procs)
    hard = t0 + deadline_s + 30.0  # the ranks' watchdogs fire at t0 + deadline_s
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
        if live and time.time() > hard:
            for q in live:
                q.kill()
            for q in live:
                q.wait()
            live = []
            rc = rc or 124
        time.sleep(0.05)
    th.join(5.0)
    if rc != 0 and not seen["line"]:
        print(json.dumps(failure_line(n, argv, f"rank processes ended with status {rc} before rank 0 reported",
                                      read_stages(stage_dir(run_id), n, t0))), flush=True)
    return rc


# ---------------------------------------------------------------------------
# stages and the watchdog (bounded, diagnosable failure)
# ---------------------------------------------------------------------------
def run_key() -> str:
    if os.environ.get("VAMPOMI_RUN_ID"):
        return os.environ["VAMPOMI_RUN_ID"]
    return "tr-{}-{}-{}".format(os.environ.get("MASTER_PORT", "0"), os.environ.get("TORCHELASTIC_RUN_ID", "none"),
                                os.environ.get("WORLD_SIZE", "1"))


def stage_dir(key: str) -> str:
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"vampomi_stages_{key}")


def read_stages(d: str, n: int, t0: float) -> dict:
    """Each rank's last reported stage (and seconds since the job start)."""
    out = {}
    for r in range(n):
        try:
            rec = json.load(open(os.path.join(d, f"rank{r}.json")))
            out[str(r)] = rec if rec.get("wall", 0) >= t0 - 5 else {"stage": "no report from this run"}
        except Exception:
            out[str(r)] = {"stage": "no report (not started?)"}
    return out


def failure_line(n: int, argv, why: str, stages: dict) -> dict:
    try:
        a = parse_args(argv)
        steps, warmup = a.steps, a.warmup
    except SystemExit:
        steps = warmup = None
    return {"metric": "VAMP iterations/s (+ achieved HBM GB/s of the A/A^T kernels)", "value": None,
            "unit": "iterations/s", "n_gpus": n, "steps": steps, "warmup": warmup, "higher_is_better": True,
            "error": why, "rank_stages": stages}


class Watchdog:
    """Stage reports of this rank (a file per rank under stage_dir) and the
    deadline: at t0 + deadline_s, rank 0 prints the failure line (unless the
    result line is out already) and every rank exits (os._exit: no Python
    teardown that could block on the device)."""

    def __init__(self, args, rank: int, world: int):
        self.rank, self.world = rank, world
        self.t0 = float(os.environ.get("VAMPOMI_BENCH_T0", time.time()))
        self.deadline = self.t0 + args.deadline_s
        self.dir = stage_dir(run_key())
        self.argv = sys.argv[1:]
        self.lock = threading.Lock()
        self.printed = False
        self.finished = False  # this rank's part of the run is complete (teardown only)
        self.partial = None  # rank 0: the finished part of the line, printed if a later phase hangs
        self.stopped = False
        os.makedirs(self.dir, exist_ok=True)
        self.stage("start")
        threading.Thread(target=self._run, daemon=True).start()

    def stage(self, what: str):
        self.cur = what
        tmp = os.path.join(self.dir, f".rank{self.rank}.{os.getpid()}")
        try:
            with open(tmp, "w") as f:
                json.dump({"stage": what, "t_s": round(time.time() - self.t0, 1), "wall": time.time(),
                           "pid": os.getpid()}, f)
            os.replace(tmp, os.path.join(self.dir, f"rank{self.rank}.json"))
        except OSError:
            pass

    def emit(self, line: dict) -> bool:
        """Print the one JSON line (rank 0), once."""
        with self.lock:
            if self.printed:
                return False
            self.printed = True
            print(json.dumps(line), flush=True)
            return True

    def stop(self):
        """The job is over (--rehearse: its rank threads have joined): no deadline action."""
        self.stopped = True

    def _run(self):
        while time.time() < self.deadline:
            if self.stopped:
                return
            time.sleep(min(1.0, max(0.05, self.deadline - time.time())))
        if self.stopped:
            return
        why = f"deadline of {self.deadline - self.t0:.0f} s passed (rank {self.rank} at stage '{self.cur}')"
        sys.stderr.write(f"bench.py rank {self.rank}: {why}\n")
        sys.stderr.flush()
        done = self.printed or (self.finished and self.rank != 0)
        if self.rank == 0 and not done:
            stages = read_stages(self.dir, self.world, self.t0)
            if self.partial is not None:
                line = dict(self.partial)
                line["error_after_result"] = why
                line["rank_stages"] = stages
            else:
                line = failure_line(self.world, self.argv, why, stages)
            self.emit(line)
            done = self.partial is not None
        os._exit(0 if done else 124)


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


CEILING_FILES = [os.path.join(ROOT, "profiles", f) for f in ("r05_hbm_read_ceiling.json", "r01h_hbm_read_ceiling.json")]


def read_ceiling(xbytes: float):
    """The measured HBM read ceiling of one MI355X (tools/hbm_ceiling: every
    byte of a buffer of about this size read once, 16-B nontemporal loads, the
    best variant's median), newest profile first: (GB/s, source) or (None, None)."""
    for f in CEILING_FILES:
        try:
            d = json.load(open(f))
        except Exception:
            continue
        sizes = {float(k[:-2]): v for k, v in d.items() if k.endswith("GB") and isinstance(v, list)}
        if not sizes:
            continue
        gb = min(sizes, key=lambda g: abs(g - xbytes / 1e9))
        best = min(sizes[gb], key=lambda v: v["us_med"])
        return best["GBs_med"], f"{os.path.relpath(f, ROOT)} ({gb:g} GB buffer, {best['variant']}, median)"
    return None, None


def same_run_ceiling(args, d, roof, n: int):
    """After the timed region, on this device: a pure read stream of the
    resident matrix (vampomi_dev_read_ceiling), the roofline's achieved rate
    against it (the same box, the same buffer; n = 1 only)."""
    if roof is None or n != 1 or args.no_read_ceiling:
        return
    try:
        c = d.read_ceiling(9)
    except Exception as e:  # noqa: BLE001  (a measurement aid: never fails the line)
        roof["read_ceiling_same_run"] = {"error": repr(e)}
        return
    roof["read_ceiling_same_run"] = {"GBs": round(c["GBs"], 1), "us_med": round(c["us_med"], 2),
                                     "bytes": int(c["bytes"]), "variant": c["variant"]}
    roof["frac_of_read_ceiling_same_run"] = round(roof["achieved"] / c["GBs"], 4)


def roofline(ks, kname: str, workload: str, period: int) -> dict:
    """The dominant kernel's achieved GB/s: algorithmic bytes per launch (exact
    count) over its average launch time (HIP events recorded in
    the dispatch packets of the sampled launches, on the stream they run on)."""
    avg_ms = ks.ms_timed / ks.timed
    bytes_per = ks.bytes_total / ks.launches
    achieved = bytes_per / (avg_ms * 1e-3) / 1e9
    traffic, tfile = pmc_traffic(kname, workload)
    ceil, cfile = read_ceiling(bytes_per)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            # the same achieved rate against what a pure read stream of the same size reaches on this hardware
            "read_ceiling_measured": round(ceil, 1) if ceil else None,
            "frac_of_read_ceiling": round(achieved / ceil, 4) if ceil else None, "read_ceiling_source": cfile,
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": int(traffic) if traffic else None,
            "traffic_unit": f"HBM bytes per launch (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, {tfile})"
            if tfile else None,
            "algorithmic_bytes_per_launch": int(bytes_per), "kernel": kname,
            "avg_launch_us": round(avg_ms * 1e3, 2), "launches": int(ks.launches), "timed_launches": int(ks.timed),
            "timing": f"HIP events in the dispatch packets of 1 in {max(1, period)} launches of each (kernel, K) "
                      "over the timed region (positions hashed from the launch index); launch counts exact"}


def cpu_baseline(y, w: dict, beta, seed: int, warmup: int, steps: int, gpu_ref_passes: float,
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


INT_MAX = 2**31 - 1


MPIEXEC = "/opt/conda/bin/mpiexec"  # the image's MPICH (hydra), which oracle/_ref/ref_data links


def ref_layouts(threads: int) -> list:
    """The reference's own decompositions of `threads` host cores: np MPI
    ranks x OMP_NUM_THREADS per rank (README.md:36-38: `mpirun -np {ranks}`
    with OMP threads per rank), np a power of two dividing `threads`."""
    out, P = [], 1
    while P <= threads:
        if threads % P == 0:
            out.append((P, threads // P))
        P *= 2
    return out


def ref_ops_time(w: dict, seed: int, threads: int) -> dict:
    """The reference's OWN data::Ax / data::ATx (src/data.cpp:294-373,
    compiled from its sources into oracle/_ref/ref_data in the build
    container) timed on a generated N x Ms matrix on `threads` host cores, in
    each of its own decompositions np x OMP (ref_layouts): np = 1 in-process,
    np > 1 under the image's MPICH `mpiexec -np`, every rank on its divide_work
    share with data::Ax's MPI_Allreduce (the job's time: the slowest rank's,
    after a barrier).  data::Ax forks an OpenMP team per marker
    (src/data.cpp:349-361), so one rank x many threads is its slowest layout.
    Returns the fastest layout's ms per call at the workload's full marker
    count (best = the smallest (5 + k) Ax + (3 + k) ATx for the caller's k, or
    the smallest Ax; chosen by the caller) with every layout's numbers.  The
    reference indexes the matrix with a 32-bit int (`i*N`, src/data.cpp:297,
    351), which overflows once a rank's M*N > 2^31 - 1 (it
    crashed with SIGSEGV at the C3 shard on one rank), so a layout whose rank
    shard would overflow is timed on the first np x floor((2^31-1)/N) markers
    and projected linearly per marker (both kernels loop over markers with
    per-marker work of N)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_data")
    if not os.path.exists(exe):
        return {"skipped": "oracle/_ref/ref_data not built (needs /root/reference in the build container)"}
    N, Mt = w["N"], w["Mt"]
    layouts, errors = [], []
    t0 = time.perf_counter()
    budget = float(os.environ.get("VAMPOMI_REF_LEG_BUDGET_S", "240"))  # the whole leg (a few s per layout at C2)
    for P, omp in ref_layouts(threads):
        left = budget - (time.perf_counter() - t0)
        if left < 10:
            errors.append(f"np={P}: skipped, the leg's {budget:.0f} s budget is spent")
            continue
        Ms = min(Mt, P * (INT_MAX // N))
        env = dict(os.environ, OMP_NUM_THREADS=str(omp))
        cmd = [exe, "time", str(N), str(Ms), "2", str(seed)]
        if P > 1:
            if not os.path.exists(MPIEXEC):
                errors.append(f"np={P}: {MPIEXEC} not found")
                continue
            cmd = [MPIEXEC, "-np", str(P)] + cmd
        try:
            out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=min(150.0, left))
        except subprocess.TimeoutExpired:
            errors.append(f"np={P}: timed out")
            continue
        lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        if out.returncode != 0 or not lines:
            errors.append(f"np={P}: exit {out.returncode}: {out.stderr[-200:]}")
            continue
        r = json.loads(lines[-1])
        # progress on stderr (a long CPU leg is not a hung run)
        print(f"[cpu reference leg] np={P} x omp={r['threads']}: Ax {r['ax_ms']:.1f} ms, ATx {r['atx_ms']:.1f} ms "
              f"on {N} x {Ms}", file=sys.stderr, flush=True)
        scale = Mt / Ms
        lay = {"np": P, "omp": r["threads"], "ax_ms": round(r["ax_ms"] * scale, 3),
               "atx_ms": round(r["atx_ms"] * scale, 3), "Ms": Ms}
        if Ms < Mt:
            lay["projected_from"] = (f"{N} x {Ms} ({P} x the largest rank shard whose M*N fits the reference's "
                                     f"32-bit int index, src/data.cpp:297,351), x {scale:.3f} per marker: Ax "
                                     f"{r['ax_ms']:.1f} ms, ATx {r['atx_ms']:.1f} ms measured")
        layouts.append(lay)
    if not layouts:
        return {"error": "; ".join(errors)}
    res = {"threads": threads, "layouts": layouts}
    if errors:
        res["layout_errors"] = errors
    return res


def _best_layout(r: dict, cost) -> dict:
    """The layout of ref_ops_time's result with the smallest cost(layout)."""
    return min(r["layouts"], key=cost)


def cpu_reference_ops(w: dict, seed: int, threads: int, k_cg: float):
    """The reference's own Ax / ATx (ref_ops_time) and its projected iteration
    rate from its own call counts per iteration (it > 1): 5 + k Ax and 3 + k
    ATx with k = k1 + k2 CG steps (src/vamp.cpp:232,303,508,518-519,653-654,
    681,826), k from the GPU window, in its fastest np x OMP
    decomposition of the same host cores (every layout reported).  The
    denoiser/EM (< 1 % of its CPU time) is left out."""
    r = ref_ops_time(w, seed, threads)
    if "layouts" not in r:
        return r

    def t_it(lay):
        return ((5 + k_cg) * lay["ax_ms"] + (3 + k_cg) * lay["atx_ms"]) * 1e-3

    b = _best_layout(r, t_it)
    one = next((lay for lay in r["layouts"] if lay["np"] == 1), None)
    out = {"value": 1.0 / t_it(b), "unit": "VAMP iterations/s", "kind": "reference", "projected": True,
           "cores": threads, "np": b["np"], "omp": b["omp"], "ax_ms": b["ax_ms"], "atx_ms": b["atx_ms"],
           "layouts": [dict(lay, it_per_s=round(1.0 / t_it(lay), 5)) for lay in r["layouts"]],
           "sample": f"Ax and ATx (mean of 2 calls each, the slowest rank's) of the reference's src/data.cpp "
                     f"(oracle/_ref) on a generated {w['N']} x {w['Mt']} matrix, {threads} host cores as np MPI "
                     f"ranks (MPICH mpiexec) x OMP threads; value = the fastest layout (np={b['np']} x "
                     f"omp={b['omp']}); iteration = (5 + k) Ax + (3 + k) ATx, k = {k_cg:.2f} (the GPU window's mean "
                     f"CG + Onsager steps)"}
    if one is not None:
        out["value_np1"] = 1.0 / t_it(one)
    for key in ("layout_errors",):
        if key in r:
            out[key] = r[key]
    if "projected_from" in b:
        out["projected_from"] = b["projected_from"]
    return out


def stated_cpu_baseline(line: dict) -> dict:
    """`cpu_baseline` states the FASTER of the two CPU measurements of the
    same host cores: the oracle port's measured iterations (one process,
    OpenMP over samples in A.x, no per-marker fork) and the reference's own
    operators in their fastest np x OMP decomposition (cpu_reference_ops);
    the other stays in the line (`cpu_port` when the reference is faster)."""
    port, ref = line.get("cpu_baseline"), line.get("cpu_reference_ops")
    if (isinstance(port, dict) and isinstance(ref, dict) and port.get("value") and ref.get("value")
            and ref["value"] > port["value"]):
        line["cpu_port"] = port
        line["cpu_baseline"] = {k: ref[k] for k in ("value", "unit", "cores", "kind", "sample", "np", "omp",
                                                     "projected", "upper_bound") if k in ref}
        line["cpu_baseline"]["why"] = "the faster of the port and the reference's own operators (cpu_reference_ops)"
    return line


def cpu_reference_ops_assoc(w: dict, seed: int, threads: int):
    """c5: of one LOO test (src/main_meth.cpp:245-264) only the reference's
    z1 = A x1_hat (data::Ax) builds here; data::pvals_loo (src/data.cpp:385-417)
    calls linear_reg1d_pvals from the Boost-dependent src/utilities.cpp.  So
    this times the reference's Ax (its fastest np x OMP layout, ref_ops_time)
    and reports the rate a test could at most reach if its per-marker pass
    were free: an UPPER bound on the reference."""
    r = ref_ops_time(w, seed, threads)
    if "layouts" not in r:
        return r
    b = _best_layout(r, lambda lay: lay["ax_ms"])
    out = {"value": w["Mt"] / (b["ax_ms"] * 1e-3), "unit": "markers/s", "kind": "reference", "projected": True,
           "upper_bound": True, "cores": threads, "np": b["np"], "omp": b["omp"], "ax_ms": b["ax_ms"],
           "layouts": r["layouts"],
           "sample": f"the reference's data::Ax (src/data.cpp:340-373, oracle/_ref) on a generated {w['N']} x "
                     f"{w['Mt']} matrix, {threads} host cores as np MPI ranks x OMP threads, the fastest (np="
                     f"{b['np']} x omp={b['omp']}): the test's A x1_hat only (pvals_loo needs Boost, absent), so "
                     "markers / Ax time bounds the reference's rate from above"}
    if "projected_from" in b:
        out["projected_from"] = b["projected_from"]
    return out


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
    return R.gather(mine)


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

    def __init__(self, timeout_s: float = 1800.0):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        import datetime

        import torch.distributed as dist

        self.dist = dist
        if self.world > 1:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=max(30.0, timeout_s)))

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

    def bcast(self, obj):
        if self.world == 1:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def gather(self, obj) -> list:
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


class Solo:
    """Ranks of a one-rank measurement inside a multi-rank job (rank 0's 1-GPU
    bases): no collectives."""
    world, rank = 1, 0
    dist = None

    def __init__(self, local: int):
        self.local = local

    def max(self, v):
        return v

    def sum(self, v):
        return v

    def barrier(self):
        pass

    def bcast(self, obj):
        return obj

    def gather(self, obj) -> list:
        return [obj]


def dry_run(args, R: Ranks, wd: Watchdog):
    """The launcher, rendezvous, barrier and max-over-ranks path without a GPU."""
    wd.stage("dry-run barrier")
    R.barrier()
    if R.rank == args.dry_run_hang_rank:
        wd.stage("dry-run hang (test)")
        while True:  # a rank that stops answering: the watchdogs must end the job
            time.sleep(3600)
    wd.stage("dry-run timed")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    R.barrier()
    el = R.max(time.perf_counter() - t0)
    seen = int(R.sum(1.0))
    wd.finished = True
    if R.rank == 0:
        wd.emit({"metric": "dry run", "value": 0.0, "unit": "none", "n_gpus": R.world, "steps": args.steps,
                 "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "ranks_seen": seen,
                 "dry_run": True})
    R.close()


def open_data(R, w: dict, device: int):
    """A context for workload w over R's ranks (an RCCL communicator if
    R.world > 1; its id made on rank 0 and broadcast over gloo)."""
    import vampomi_amd as va

    comm_id = R.bcast(va.comm_unique_id() if R.rank == 0 else None) if R.world > 1 else None
    return va.Data(w["N"], w["Mt"], rank=R.rank, nranks=R.world, comm_id=comm_id, device=device)


def vamp_window(args, R, w: dict, wd: Watchdog, steps: int, warmup: int, tag: str, keep=False) -> dict:
    """Generate workload w on the device, run `warmup` untimed and `steps`
    timed VAMP iterations over R's ranks; returns the measurements (and,
    with keep, the open context and run for the caller's further legs)."""
    import torch

    import vampomi_amd as va

    wd.stage(f"{tag}: open {w['workload']} (N={w['N']}, Mt={w['Mt']}, {R.world} rank(s))")
    d = open_data(R, w, R.local)
    try:
        wd.stage(f"{tag}: generate")
        t0 = time.perf_counter()
        d.generate(args.seed, w["kind"])
        model = w.get("model", "linear")
        if model == "bin_class":
            beta = d.simulate_phen_binary(args.seed + 1, lam=0.1, h2=0.8)
        else:
            beta = d.simulate_phen(args.seed + 1, lam=0.1, h2=0.8)
        t_setup = time.perf_counter() - t0
        if args.op_variant is not None:
            d.set_variant(3, args.op_variant)
        opts = va.VampOptions(max_iter=warmup + steps, stop_criteria_thr=0.0, batch_rhs=args.batch_rhs, model=model)
        v = va.Vamp(d, opts, true_signal=beta)
        wd.stage(f"{tag}: warmup ({warmup} iterations)")
        v.begin()
        for _ in range(warmup):
            v.step()
        ref0, _ = v.a_passes
        d.reset_stats()
        d.set_timing(not args.no_timing, args.timing_period)

        def barrier():
            d.sync()
            torch.cuda.synchronize() if torch.cuda.is_available() else None
            R.barrier()

        wd.stage(f"{tag}: timed ({steps} iterations)")
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            v.step()
        barrier()
        el = R.max(time.perf_counter() - t0)
        st = d.stats()
        ref1, _ = v.a_passes
        res = {"el": el, "st": st, "summ": v.summary(), "ref_passes": (ref1 - ref0) / steps, "setup": t_setup,
               "M": d.M, "nranks": d.nranks, "steps": steps, "warmup": warmup, "model": model, "beta": beta,
               "opts": opts, "barrier": barrier}
        res["rank_times"] = per_rank_times(R, st, el)
        v.end()
        if keep:
            res["d"] = d
            d = None
        return res
    finally:
        if d is not None:
            wd.stage(f"{tag}: close")
            d.close()


def dominant_roofline(args, res: dict, w: dict, kernel_name) -> dict:
    """roofline of the (kernel class, K) with the most device time."""
    st = res["st"]
    cands = []
    for which, arr in ((0, st.ax_k), (1, st.atx_k), (3, st.op_k)):
        for k in range(4):
            if arr[k].timed:
                cands.append((arr[k].ms_total, which, k + 1, arr[k]))
    if not cands:
        return None
    _, which, K, ks = max(cands, key=lambda c: c[0])
    # A^T.u in the CG carries the lmmse_mult epilogue (mode 1); the one-pass
    # operator's instantiation depends on N (passed as mode)
    return roofline(ks, kernel_name(which, K, w["N"] if which == 3 else 1), w["workload"], args.timing_period)


def summary_of(res: dict, w: dict, strong: bool, n: int) -> dict:
    """A compact record of one vamp_window (1-GPU bases, the headline phase)."""
    st, el, steps = res["st"], res["el"], res["steps"]
    all_ms = st.ax.ms_total + st.atx.ms_total + st.op.ms_total
    all_bytes = st.ax.bytes_total + st.atx.bytes_total + st.op.bytes_total
    it_s = steps / el
    return {"workload": w["workload"], "N": w["N"], "Mt": w["Mt"], "M_per_gpu": res["M"], "n_gpus": n,
            "iterations_timed": f"{res['warmup'] + 1}-{res['warmup'] + steps}",
            "iterations_per_s": round(it_s, 4), "value": round(it_s if (strong or n == 1) else n * it_s, 4),
            "ms_per_step": round(el / steps * 1e3, 3), "passes_exec_per_step": round(st.a_passes_exec / steps, 2),
            "hbm_gbs_all_A_kernels": round(all_bytes / (all_ms * 1e-3) / 1e9, 1) if all_ms > 0 else None,
            "a_kernel_frac_of_step": round(all_ms * 1e-3 / el, 4) if el > 0 else None,
            "cg_iters": res["summ"]["cg_iters"][res["warmup"]:], "ons_iters": res["summ"]["ons_iters"][res["warmup"]:],
            "setup_s": round(res["setup"], 2)}


def per_pass_marker_ms(rec: dict) -> float:
    """ms per executed pass over X per marker (a 1-GPU basis at another Mt)."""
    return rec["ms_per_step"] / (rec["passes_exec_per_step"] * rec["M_per_gpu"])


def one_gpu_bases(args, R: Ranks, wd: Watchdog, w: dict, headline: bool) -> dict:
    """Rank 0 alone, on its own GPU, before any n-rank context exists (the
    other ranks wait at a gloo barrier): the 1-GPU runs the n-rank line is read
    against, measured in this job on this node.
      same_problem: the n-rank workload's WHOLE problem on one GPU, when it
        fits (c2-weak: 4n GB): the same iterations, so speedup = this run's
        iterations/s over it, exactly;
      c3big: N = 100,000 x 300,000 (240 GB, the most of configs[2] one
        MI355X holds), for the headline configs[2] phase (400 GB, which no
        single GPU holds): its ms per executed pass per marker, times the
        headline's markers and passes, is the 1-GPU equivalent."""
    out = {}
    if R.rank == 0:
        solo = Solo(R.local)
        if w["N"] * w["Mt"] * 8 <= 200e9:
            wd.stage("basis: same problem on 1 GPU")
            try:
                r = vamp_window(args, solo, dict(w, workload=w["workload"] + "@1gpu"), wd, args.steps, args.warmup,
                                "basis same-problem")
                out["same_problem"] = summary_of(r, w, True, 1)
            except Exception as e:
                traceback.print_exc()
                out["same_problem"] = {"error": repr(e)}
        if headline:
            wb = get_workload("c3big", 1)
            try:
                r = vamp_window(args, solo, wb, wd, 4, 1, "basis c3big")
                rec = summary_of(r, wb, False, 1)
                rec["ms_per_pass_per_marker"] = per_pass_marker_ms(rec)
                out["c3big"] = rec
            except Exception as e:
                traceback.print_exc()
                out["c3big"] = {"error": repr(e)}
    wd.stage("basis: barrier")
    R.barrier()
    return out


def run_linear(args, R: Ranks, wd: Watchdog, w: dict, t_start: float) -> dict:
    """The linear / probit VAMP line of workload w on R's ranks."""
    import vampomi_amd as va

    n = R.world
    strong = w.get("scaling") == "strong"
    auto_multi = args.config == "auto" and n > 1
    headline = auto_multi and not args.no_headline
    bases = one_gpu_bases(args, R, wd, w, headline or (strong and w["workload"] == "c3full")) if n > 1 else {}

    res = vamp_window(args, R, w, wd, args.steps, args.warmup, "main", keep=True)
    d, st, el, model = res["d"], res["st"], res["el"], res["model"]
    try:
        roof = dominant_roofline(args, res, w, d.kernel_name)
        same_run_ceiling(args, d, roof, n)
        y = d.get_phen() if (R.rank == 0 and n == 1 and not args.no_cpu_baseline) else None
        with_writes = (write_rate(args, d, R, res["opts"], res["beta"], res["barrier"], el) if args.write else None)
    finally:
        wd.stage("main: close")
        d.close()
    it_s = args.steps / el
    all_ms = st.ax.ms_total + st.atx.ms_total + st.op.ms_total
    all_bytes = st.ax.bytes_total + st.atx.bytes_total + st.op.bytes_total
    line = {
        "metric": "VAMP iterations/s (+ achieved HBM GB/s of the A/A^T kernels)",
        "value": round(it_s if strong else n * it_s, 4),
        "unit": "iterations/s" if (strong or n == 1) else "shard-iterations/s",
        "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (index-keyed dyadic generator, generated in HBM)",
        "config": {"workload": w["workload"], "model": model, "N": w["N"], "Mt": w["Mt"], "M_per_gpu": res["M"],
                   "design": "gaussian" if w["kind"] == va.GEN_GAUSS else "methylation-like",
                   "iterations_timed": f"{args.warmup + 1}-{args.warmup + args.steps}",
                   "parallelism": f"markers sharded over {n} GPU(s)" + (", RCCL all-reduce" if n > 1 else ""),
                   "comm": {"backend": ("loopback" if os.environ.get("VAMPOMI_COMM") == "loopback" else "rccl")
                            if n > 1 else "none", "nranks": res["nranks"]}},
        "roofline": roof,
        "hbm_gbs_all_A_kernels": round(all_bytes / (all_ms * 1e-3) / 1e9, 1) if all_ms > 0 else None,
        "passes_exec_per_step": round(st.a_passes_exec / args.steps, 2),  # stats reset at the timed region
        "passes_ref_per_step": round(res["ref_passes"], 2),
        # device time of the A-kernels over the wall time: each (kernel, K)'s
        # average over its sampled launches (hashed positions, unbiased over the
        # solve's steps) times its exact launch count; --timing-period 1 times
        # every launch (a measured sum, at 1-2.6 % of the iteration rate)
        "a_kernel_frac_of_step": round(all_ms * 1e-3 / el, 4) if el > 0 else None,
        "a_kernel_timing": {"timed_launches": int(st.ax.timed + st.atx.timed + st.op.timed),
                            "launches": int(st.ax.launches + st.atx.launches + st.op.launches),
                            "period": args.timing_period},
        "per_rank": res["rank_times"],
        "cg_iters": res["summ"]["cg_iters"][args.warmup:], "ons_iters": res["summ"]["ons_iters"][args.warmup:],
        "setup_s": round(res["setup"], 2),
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
    if n > 1:
        line["scaling_basis"] = (
            "read against the n = 1 line of the same workload family: `python bench.py --gpus 1` (c2, configs[1]: "
            "N = 10,000 x 50,000, the same per-GPU shard as c2-weak)" if w["workload"] == "c2-weak" else
            "one_gpu.c3big (measured in this job; configs[2] does not fit one GPU)" if strong else
            f"the n = 1 line of --config {args.config}")
        one = {}
        if "same_problem" in bases:
            sp = bases["same_problem"]
            one["same_problem"] = sp
            if "iterations_per_s" in sp:
                one["same_problem"]["speedup_of_this_run"] = round(it_s / sp["iterations_per_s"], 4)
                one["same_problem"]["note"] = (f"the whole {w['N']} x {w['Mt']} problem of this line on rank 0's GPU "
                                               "alone, same iterations: strong scaling of this exact problem")
        if "c3big" in bases:
            one["c3big"] = bases["c3big"]
        if one:
            line["one_gpu"] = one
        if strong and "c3big" in bases and "ms_per_pass_per_marker" in bases["c3big"]:
            line["one_gpu_equivalent"] = equivalent(bases["c3big"], w["Mt"], line["passes_exec_per_step"], it_s, n)
    wd.partial = line  # a hang in a later phase still reports this
    if headline:
        line["headline_c3full"] = run_headline(args, R, wd, bases.get("c3big"))
        wd.partial = line
    if model == "bin_class":
        line["parity_note"] = ("probit: x1_hat/r1 parity bar is max(1e-10, k x the oracle's own rank-count spread), "
                               "integers exact (DESIGN.md §3)")
    if R.rank == 0 and n == 1 and not args.no_cpu_baseline:
        wd.stage("cpu baseline")
        if w["workload"] == "c3big":
            # the oracle's leg would generate the whole 240 GB matrix on the host
            line["cpu_baseline"] = {"skipped": "240 GB matrix; see the --config c3 line (same N, 62,500-marker shard)"}
        else:
            try:
                line["cpu_baseline"] = cpu_baseline(y, w, res["beta"], args.seed, args.warmup, args.steps,
                                                    res["ref_passes"], args.cpu_budget)
            except Exception as e:  # reported, never fatal for the GPU number
                line["cpu_baseline"] = {"error": repr(e)}
        if model == "linear":
            try:
                k_cg = (sum(line["cg_iters"]) + sum(line["ons_iters"])) / max(len(line["cg_iters"]), 1)
                threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
                line["cpu_reference_ops"] = cpu_reference_ops(w, args.seed, threads, k_cg)
            except Exception as e:
                line["cpu_reference_ops"] = {"error": repr(e)}
            line = stated_cpu_baseline(line)
    line["wall_s_since_start"] = round(time.perf_counter() - t_start, 1)
    return line


def equivalent(c3big: dict, Mt: int, passes: float, it_s: float, n: int) -> dict:
    """The 1-GPU iterations/s of an Mt-marker problem at N = 100,000 from the
    measured c3big basis: its ms per executed pass per marker x Mt x this
    run's executed passes per iteration (no single MI355X holds the problem)."""
    one = 1e3 / (c3big["ms_per_pass_per_marker"] * Mt * passes)
    return {"value": round(one, 4), "unit": "iterations/s", "measured_in_this_job": True,
            "source": f"one_gpu.c3big (N = 100,000 x 300,000 on rank 0's GPU alone, {c3big['ms_per_step']} ms per "
                      f"iteration at {c3big['passes_exec_per_step']} passes) x Mt = {Mt} x this run's {passes} passes "
                      "per iteration; the problem itself does not fit one GPU",
            "strong_scaling_efficiency": round(it_s / (n * one), 4)}


def run_headline(args, R: Ranks, wd: Watchdog, c3big) -> dict:
    """configs[2] itself (N = 100,000 x Mt = 500,000, 400 GB) sharded over
    this job's ranks, after the main phase: north_star's headline problem at
    n = 2 / 4 / 8 (it does not fit one GPU).  Fewer timed iterations (at most
    10) keep the job short; errors are recorded, not fatal for the line."""
    w = get_workload("c3full", R.world)
    steps = min(args.steps, 10)
    try:
        res = vamp_window(args, R, w, wd, steps, args.warmup, "headline", keep=True)
        d = res["d"]
        try:
            roof = dominant_roofline(args, res, w, d.kernel_name)
        finally:
            d.close()
        rec = summary_of(res, w, True, R.world)
        rec["roofline"] = roof
        rec["per_rank"] = res["rank_times"]
        if c3big and "ms_per_pass_per_marker" in c3big:
            rec["one_gpu_equivalent"] = equivalent(c3big, w["Mt"], rec["passes_exec_per_step"],
                                                   rec["iterations_per_s"], R.world)
        return rec
    except Exception as e:
        return {"error": repr(e), "workload": "c3full"}


def bench_assoc(args, R: Ranks, wd: Watchdog, w: dict, t_start):
    """--config c5: the LOO association test (src/main_meth.cpp:245-264) on
    device-resident inputs; a step is one whole test."""
    import ctypes as C

    import numpy as np
    import torch

    import vampomi_amd as va

    N, Mt = w["N"], w["Mt"]
    wd.stage("c5: open + generate")
    d = open_data(R, w, R.local)
    d.generate(args.seed, w["kind"])
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

    wd.stage("c5: warmup")
    for _ in range(args.warmup):
        step()
    d.reset_stats()
    d.set_timing(not args.no_timing, args.timing_period)

    def barrier():
        d.sync()
        torch.cuda.synchronize()
        R.barrier()

    wd.stage("c5: timed")
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
        same_run_ceiling(args, d, roof, R.world)
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
        wd.stage("cpu baseline")
        try:
            line["cpu_baseline"] = cpu_baseline_assoc(d, w, est, args.seed)
        except Exception as e:
            line["cpu_baseline"] = {"error": repr(e)}
        try:
            threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
            line["cpu_reference_ops"] = cpu_reference_ops_assoc(w, args.seed, threads)
        except Exception as e:
            line["cpu_reference_ops"] = {"error": repr(e)}
        line = stated_cpu_baseline(line)
    d.close()
    return line


class ThreadRanks:
    """Ranks of a --rehearse job: P threads of this process, one loopback rank
    each, all on GPU 0 (the interface of Ranks: max / sum / barrier / bcast,
    combined in rank order)."""

    class Shared:
        def __init__(self, P: int, timeout_s: float):
            self.P = P
            self.bar = threading.Barrier(P, timeout=timeout_s)
            self.vals = [None] * P

    dist = None

    def __init__(self, shared: "ThreadRanks.Shared", rank: int):
        self.s, self.rank, self.world, self.local = shared, rank, shared.P, 0

    def _combine(self, v, fn):
        self.s.vals[self.rank] = v
        self.s.bar.wait()
        out = fn(list(self.s.vals))
        self.s.bar.wait()
        return out

    def max(self, v: float) -> float:
        return self._combine(v, max)

    def sum(self, v: float) -> float:
        return self._combine(v, lambda a: float(sum(a)))

    def barrier(self):
        self.s.bar.wait()

    def bcast(self, obj):
        return self._combine(obj, lambda a: a[0])

    def gather(self, obj) -> list:
        return self._combine(obj, list)

    def close(self):
        pass


def rehearse(args) -> int:
    """--rehearse P: the whole n > 1 flow of `bench.py --gpus P` (rank 0's
    1-GPU bases, the main phase, the configs[2] headline phase, the line) with
    P loopback ranks as threads on GPU 0 and every workload's markers scaled
    by --rehearse-scale, so that the driver's first multi-GPU run is not the
    first time this code path runs on the device.  Prints rank 0's line with
    "rehearsal" set; its rates are one GPU's, not a scaling result."""
    global WORKLOAD_SCALE
    WORKLOAD_SCALE = args.rehearse_scale
    os.environ["VAMPOMI_COMM"] = "loopback"
    os.environ.setdefault("VAMPOMI_RUN_ID", f"rehearse-{os.getpid()}")
    P = args.rehearse
    args.gpus = P
    import torch  # noqa: F401  (before libvampomi: one HIP runtime per process)

    shared = ThreadRanks.Shared(P, args.deadline_s)
    lines, errs = [None] * P, []
    t_start = time.perf_counter()

    wds = [None] * P

    def work(r):
        R = ThreadRanks(shared, r)
        wd = wds[r] = Watchdog(args, r, P)
        try:
            w = get_workload(args.config, P)
            lines[r] = run_linear(args, R, wd, w, t_start) if w.get("model") != "loo" else \
                bench_assoc(args, R, wd, w, t_start)
            wd.finished = True
        except BaseException as e:  # noqa: BLE001 - reported in the line
            traceback.print_exc()
            errs.append((r, repr(e)))
            shared.bar.abort()  # the other ranks' next barrier fails instead of waiting

    th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(P)]
    [t.start() for t in th]
    [t.join() for t in th]
    for wd in wds:
        if wd is not None:
            wd.stop()
    line = lines[0] or failure_line(P, sys.argv[1:], f"rehearsal: {errs}", {})
    line["rehearsal"] = {"loopback_rank_threads_on_one_gpu": P, "markers_scale": args.rehearse_scale,
                         "errors": errs,
                         "note": "the n > 1 flow on one GPU; rates are not multi-GPU numbers"}
    print(json.dumps(line), flush=True)
    return 0 if (lines[0] is not None and not errs) else 1


def main():
    args = parse_args()
    if args.rehearse > 0:
        sys.exit(rehearse(args))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # start the ranks before this process touches the GPU (or imports torch)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], args.deadline_s))
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    wd = Watchdog(args, rank, world)
    # bounded RCCL (engine.cpp): creation and every collective fail with a
    # status instead of waiting for a peer that never comes
    os.environ.setdefault("VAMPOMI_COMM_INIT_TIMEOUT_S", "90")
    os.environ.setdefault("VAMPOMI_COLL_TIMEOUT_S", "120")
    t_start = time.perf_counter()
    wd.stage("import torch")
    import torch  # noqa: F401  (before libvampomi: one HIP runtime per process)

    wd.stage("gloo rendezvous")
    R = Ranks(timeout_s=args.deadline_s)
    try:
        if args.dry_run:
            return dry_run(args, R, wd)
        if args.gpus != R.world:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={R.world}: launch one process per GPU")

        if torch.cuda.is_available():
            # one GPU per local rank; more ranks than visible GPUs share them
            # modulo (RCCL then refuses the job at creation: "Duplicate GPU",
            # reported in the line like any other failure)
            R.local = R.local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(R.local)  # torch's own context on this rank's GPU, not on GPU 0
        w = get_workload(args.config, R.world)
        if w.get("model") == "loo":
            line = bench_assoc(args, R, wd, w, t_start)
        else:
            line = run_linear(args, R, wd, w, t_start)
        wd.finished = True
        if R.rank == 0:
            wd.emit(line)
        wd.stage("done")
    except SystemExit:
        raise
    except BaseException as e:  # one diagnosable line instead of a bare traceback
        traceback.print_exc()
        wd.stage(f"failed: {e!r}"[:300])
        if R.rank == 0:
            time.sleep(1.0)  # let the other ranks record where they are
            line = wd.partial
            if line is not None:
                line = dict(line, error_after_result=repr(e))
            else:
                line = failure_line(R.world, sys.argv[1:], f"rank 0: {e!r}", read_stages(wd.dir, R.world, wd.t0))
            wd.emit(line)
        else:
            time.sleep(5.0)  # rank 0 prints the line (with every rank's stage) before this rank's exit ends the job
        sys.stdout.flush()
        os._exit(0 if (R.rank == 0 and wd.partial is not None) else 1)
    R.close()


if __name__ == "__main__":
    main()
