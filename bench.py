"""bench.py — VAMP iterations/s + HBM GB/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c3big|c4|c4full|c5] [--no-cpu-baseline]

A "step" is one VAMP iteration (src/vamp.cpp:148-428) of the linear model
(or src/vamp_probit.cpp:68-463 of the probit model for c4)
over the whole synthetic problem, with every vector and the fp64 design
matrix already resident in HBM.  --stop-criteria-thr is 0, so exactly W+K
iterations run; W are untimed.

Workloads (synthetic, generated on the device):
  c2 (default)  N=10,000 x Mt=50,000 i.i.d. Gaussian design (BASELINE configs[1]);
                with --gpus n > 1: weak scaling over markers (the reference's
                own sharding): N = 10,000, Mt = 50,000*n, 4 GB per GPU.
  c3            per-GPU shard of configs[2] (N=100,000 x 62,500 markers per GPU,
                methylation-like); at n=8 it is N=100,000 x Mt=500,000.
  c4            probit model (configs[3], src/vamp_probit.cpp): N=50,000 x 50,000
                markers per GPU, binary phenotype; at n=4 it is N=50,000 x Mt=200,000.
  c4full        configs[3] whole on any n (80 GB: fits one MI355X).
  c5            LOO association test (configs[4]): N=100,000 x 62,500 methylation-
                like markers per GPU; at n=8 it is N=100,000 x Mt=500,000.  A step
                is one whole test (A.x of the estimate, then the per-marker pass
                and the p-values); value = markers tested per second.

value = n_gpus * iterations/s ("shard-iterations/s": VAMP iterations over one
GPU's shard; at n=1 exactly iterations/s of the workload).  Multi-GPU: one
process per GPU (torchrun), RCCL communicator inside libvampomi for the data
path, torch.distributed (gloo) only for the id broadcast, barriers and the
max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before libvampomi: one HIP runtime)
import torch.distributed as dist  # noqa: E402

import vampomi_amd as va  # noqa: E402
from vampomi_amd.workloads import workload  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PMC_FILE = os.path.join(ROOT, "profiles", "r01_pmc_traffic_{}.json")


def pmc_traffic(kernel: str, workload: str):
    """HBM bytes per launch of `kernel` on `workload` from the committed
    rocprofv3 --pmc summary (tools/pmc.sh: FETCH_SIZE x2 gfx950 correction +
    WRITE_SIZE); None when that workload was not profiled."""
    try:
        import json as _j

        for name, d in _j.load(open(PMC_FILE.format(workload))).items():
            if kernel in name:
                return d.get("traffic_bytes_per_launch")
    except Exception:
        return None
    return None


def cpu_baseline(d: "va.Data", w: dict, beta: np.ndarray, seed: int, budget_s: float = 20.0) -> dict:
    """The CPU oracle (C restatement, OpenMP) on a bounded sample of the same workload."""
    from oracle import pyoracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    N, Mt = w["N"], w["Mt"]
    t0 = time.perf_counter()
    X = O.generate_markers(seed, w["kind"], N, 0, Mt)  # bit-identical to the device shard
    tgen = time.perf_counter() - t0
    y = d.get_phen()
    # two iterations first to size the sample (iteration 1 of the probit model
    # is a single CG step, unrepresentative alone), then a fresh run of k
    t0 = time.perf_counter()
    model = w.get("model", "linear")
    r1 = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=2, stop_criteria_thr=0.0, keep_hist=False, model=model)
    t1 = (time.perf_counter() - t0) / 2
    k = max(2, min(10, int(budget_s / max(t1, 1e-3))))
    if k > 2:
        t0 = time.perf_counter()
        r = O.vamp_infere(X, y, Mt, true_signal=beta, max_iter=k, stop_criteria_thr=0.0, keep_hist=False,
                          model=model)
        tk = time.perf_counter() - t0
    else:
        r, tk = r1, 2 * t1
    passes = int(r["a_passes"])
    return {
        "value": k / tk,
        "unit": "VAMP iterations/s",
        "cores": threads,
        "kind": "port",
        "sample": f"iterations 1-{k} of {w['workload']} (N={N}, Mt={Mt}) on {threads} OpenMP threads; "
                  f"{passes} A/A^T passes = {passes * 8.0 * N * Mt / tk / 1e9:.1f} GB/s effective; "
                  f"data generation ({tgen:.1f} s) not timed",
        "cg_iters": [int(a) for a in r["cg_iters"]],
        "ons_iters": [int(a) for a in r["ons_iters"]],
    }


def cpu_baseline_assoc(d: "va.Data", w: dict, est: np.ndarray, seed: int) -> dict:
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


def bench_assoc(args, d, w, world, rank, t_start):
    """--config c5: the LOO association test (src/main_meth.cpp:245-264) on
    device-resident inputs; a step is one whole test."""
    import ctypes as C

    N, Mt = w["N"], w["Mt"]
    beta = d.simulate_phen(args.seed + 1, lam=0.1, h2=0.5)
    t_setup = time.perf_counter() - t_start
    est = beta * 0.9 / np.sqrt(N)  # an estimate file's values (x1_hat / sqrt(N))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
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
        if world > 1:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    el = time.perf_counter() - t0
    st = d.stats()
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    roof = None
    if st.loo.launches:
        ks = st.loo
        kname = va.kernel_name(2, 1, 0)
        avg_ms = ks.ms_total / ks.launches
        bytes_per = ks.bytes_total / ks.launches
        achieved = bytes_per / (avg_ms * 1e-3) / 1e9
        traffic = pmc_traffic(kname, w["workload"])
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": int(traffic) if traffic else None,
                "traffic_unit": "HBM bytes per launch (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
                                f"profiles/{os.path.basename(PMC_FILE.format(w['workload']))})",
                "algorithmic_bytes_per_launch": int(bytes_per), "kernel": kname,
                "avg_launch_us": round(avg_ms * 1e3, 2), "launches": int(ks.launches),
                "ax_avg_launch_us": round(st.ax.ms_total / max(st.ax.launches, 1) * 1e3, 2)}
    line = {
        "metric": "LOO association test: markers tested/s (+ achieved HBM GB/s of the per-marker pass)",
        "value": round(Mt * args.steps / el, 1),
        "unit": "markers/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (index-keyed dyadic generator, generated in HBM)",
        "config": {"workload": w["workload"], "model": "association_test loo", "N": N, "Mt": Mt, "M_per_gpu": d.M,
                   "design": "methylation-like", "parallelism": f"markers sharded over {world} GPU(s)"},
        "roofline": roof,
        "setup_s": round(t_setup, 2),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline_assoc(d, w, est, args.seed)
        except Exception as e:
            line["cpu_baseline"] = {"error": repr(e)}
    d.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c3big", "c4", "c4full", "c5"])
    ap.add_argument("--seed", type=int, default=20250711)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event kernel timing")
    ap.add_argument("--timing-period", type=int, default=4,
                    help="time one A/A^T launch in this many of each (kernel, K) with HIP events")
    ap.add_argument("--batch-rhs", type=int, default=4)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)  # torch's own context on this rank's GPU, not on GPU 0
    n = world
    if world > 1:
        dist.init_process_group("gloo")
    w = workload(args.config, n)
    N, Mt = w["N"], w["Mt"]

    comm_id = None
    if world > 1:
        obj = [va.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    d = va.Data(N, Mt, rank=rank, nranks=world, comm_id=comm_id, device=local)
    t0 = time.perf_counter()
    d.generate(args.seed, w["kind"])
    model = w.get("model", "linear")
    if model == "loo":
        return bench_assoc(args, d, w, world, rank, t0)
    if model == "bin_class":
        beta = d.simulate_phen_binary(args.seed + 1, lam=0.1, h2=0.8)
    else:
        beta = d.simulate_phen(args.seed + 1, lam=0.1, h2=0.8)
    t_setup = time.perf_counter() - t0

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
        if world > 1:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        v.step()
    barrier()
    el = time.perf_counter() - t0
    st = d.stats()
    ref1, _ = v.a_passes
    summ = v.summary()
    v.end()
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    it_s = args.steps / el
    # dominant kernel: the (class, batch width) with the most device time
    cands = []
    for which, arr in ((0, st.ax_k), (1, st.atx_k), (3, st.op_k)):
        for k in range(4):
            if arr[k].launches:
                cands.append((arr[k].ms_total, which, k + 1, arr[k]))
    roof = None
    if cands:
        ms, which, K, ks = max(cands, key=lambda c: c[0])
        # A^T.u in the CG carries the lmmse_mult epilogue (mode 1); the one-pass
        # operator's instantiation depends on N (passed as mode)
        kname = va.kernel_name(which, K, N if which == 3 else 1)
        avg_ms = ks.ms_total / ks.launches
        bytes_per = ks.bytes_total / ks.launches
        achieved = bytes_per / (avg_ms * 1e-3) / 1e9
        traffic = pmc_traffic(kname, w["workload"])
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": int(traffic) if traffic else None,
                "traffic_unit": "HBM bytes per launch (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
                                f"profiles/{os.path.basename(PMC_FILE.format(w['workload']))})",
                "algorithmic_bytes_per_launch": int(bytes_per),
                "kernel": kname, "avg_launch_us": round(avg_ms * 1e3, 2), "launches": int(ks.launches),
                "timed_launches": int(ks.launches) // max(1, args.timing_period),
                "timing": f"HIP events in the dispatch packets of 1 in {max(1, args.timing_period)} launches "
                          "of each (kernel, K) over the timed region"}
    all_ms = st.ax.ms_total + st.atx.ms_total + st.op.ms_total
    all_bytes = st.ax.bytes_total + st.atx.bytes_total + st.op.bytes_total
    line = {
        "metric": "VAMP iterations/s (+ achieved HBM GB/s of the A/A^T kernels)",
        "value": round(n * it_s, 4),
        "unit": "shard-iterations/s" if n > 1 else "iterations/s",
        "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (index-keyed dyadic generator, generated in HBM)",
        "config": {"workload": w["workload"], "model": model, "N": N, "Mt": Mt, "M_per_gpu": d.M,
                   "design": "gaussian" if w["kind"] == va.GEN_GAUSS else "methylation-like",
                   "iterations_timed": f"{args.warmup + 1}-{args.warmup + args.steps}",
                   "parallelism": f"markers sharded over {n} GPU(s), RCCL all-reduce"},
        "roofline": roof,
        "hbm_gbs_all_A_kernels": round(all_bytes / (all_ms * 1e-3) / 1e9, 1) if all_ms > 0 else None,
        "passes_exec_per_step": round(st.a_passes_exec / args.steps, 2),  # stats reset at the timed region
        "passes_ref_per_step": round((ref1 - ref0) / args.steps, 2),
        "a_kernel_frac_of_step": round(all_ms * 1e-3 / el, 3) if el > 0 else None,
        "cg_iters": summ["cg_iters"][args.warmup:], "ons_iters": summ["ons_iters"][args.warmup:],
        "setup_s": round(t_setup, 2),
        "cpu_baseline": None,
    }
    if rank == 0 and n == 1 and not args.no_cpu_baseline and w["workload"] == "c3big":
        # the oracle's leg generates the whole matrix on the host (240 GB): the
        # c3 line carries the CPU baseline for the same samples and marker kind
        line["cpu_baseline"] = {"skipped": "240 GB matrix; see the --config c3 line (same N, 62,500-marker shard)"}
    elif rank == 0 and n == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(d, w, beta, args.seed)
        except Exception as e:  # reported, never fatal for the GPU number
            line["cpu_baseline"] = {"error": repr(e)}
    d.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
