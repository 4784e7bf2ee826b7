"""main_meth.exe as SEVERAL PROCESSES, the drop-in for `mpirun -np P
main_meth.exe` (src/main_meth.cpp:12-36), on one GPU:
ranks from VAMPOMI_RANK / VAMPOMI_NRANKS, the communicator id handed over by
the rendezvous file, the test-only cross-process communicator
(VAMPOMI_COMM=shm, vampomi_amd/csrc/shmcomm.cpp: RCCL refuses two ranks on one
device) in place of RCCL, every rank writing its shard of the _it_K.bin files
at S*8 (src/utilities.cpp:241-249) and rank 0 the CSV rows (:366-401).

* P processes give byte for byte the files of P loopback rank threads in one
  process (the same shards, the same rank-ordered sums): the multi-process
  path adds nothing to the arithmetic, and the loopback runs are held to the
  single-rank run and the oracle elsewhere (tests/test_gpu_sharded.py);
* against the one-process CLI: the same counts, x1_hat within 1e-10 (linear);
* a rank killed mid-run ends every process with a non-zero exit status within
  VAMPOMI_COLL_TIMEOUT_S (the survivor sees the peer gone at its next
  collective and fails instead of waiting).
"""
import os
import re
import signal
import subprocess
import threading
import time

import numpy as np
import pytest

from conftest import relerr
from _data import make_problem

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")


def _inputs(tmp, N, Mt, binary=False, seed=3):
    X, y, beta = make_problem(N, Mt, seed=seed)
    if binary:
        y = (y > 0).astype(np.float64)
    Xp, yp, tp = os.path.join(tmp, "ex.bin"), os.path.join(tmp, "ex.phen"), os.path.join(tmp, "ex_ts.bin")
    X.astype("<f8").tofile(Xp)
    with open(yp, "w") as f:
        for i, v in enumerate(y):
            f.write("%d %d %0.10f\n" % (i, i, v))  # simulation/data_sim.py:68
    beta.astype("<f8").tofile(tp)
    return Xp, yp, tp


def _cli(Xp, yp, tp, N, Mt, out, its, model):
    return [va.CLI_PATH, "--meth-file", Xp, "--phen-file", yp, "--N", str(N), "--Mt", str(Mt), "--out-dir", str(out),
            "--out-name", "ex", "--iterations", str(its), "--stop-criteria-thr", "0", "--true-signal-file", tp,
            "--model", model]


def _launch(cmd, P, tmp, tag, extra_env=None):
    """P processes of cmd (ranks 0..P-1), stdout/stderr to files; returns the Popen objects and the log paths."""
    rdzv = os.path.join(tmp, f".{tag}.rdzv")
    procs, logs = [], []
    for r in range(P):
        # VAMPOMI_RUN_ID: the job's id (as mpirun / torchrun / slurm give one): the rendezvous needs no
        # 3 s settling of the id file; VAMPOMI_COMM_INIT_TIMEOUT_S bounds the join
        env = dict(os.environ, VAMPOMI_RANK=str(r), VAMPOMI_NRANKS=str(P), VAMPOMI_COMM="shm", VAMPOMI_RDZV=rdzv,
                   VAMPOMI_COLL_TIMEOUT_S="60", VAMPOMI_COMM_INIT_TIMEOUT_S="60", VAMPOMI_RUN_ID=f"{tag}-{os.getpid()}")
        env.update(extra_env or {})
        log = os.path.join(tmp, f"{tag}_rank{r}.log")
        logs.append(log)
        with open(log, "w") as fh:
            procs.append(subprocess.Popen(cmd, stdout=fh, stderr=subprocess.STDOUT, env=env))
    return procs, logs


def _wait(procs, timeout):
    deadline = time.monotonic() + timeout
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(max(0.1, deadline - time.monotonic())))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    return rcs


def _counts(log):
    txt = open(log).read()
    return [(int(a), int(b), int(c)) for a, b, c in
            re.findall(r"it (\d+): CG iterations (\d+), onsager CG iterations (\d+)", txt)]


def _loopback(N, Mt, P, Xp, yp, tp, out, its, model):
    """The same job as P rank threads of this process (VAMPOMI_COMM=loopback), files into out."""
    cid = os.urandom(va.UNIQUE_ID_BYTES)
    beta = np.fromfile(tp, dtype="<f8")
    errs = []
    old = os.environ.get("VAMPOMI_COMM")
    os.environ["VAMPOMI_COMM"] = "loopback"

    def work(r):
        try:
            with va.Data(N, Mt, rank=r, nranks=P, comm_id=cid, device=0) as d:
                d.read_phen(yp, standardize=model == "linear")
                d.read_methylation_data(Xp)
                v = va.Vamp(d, va.VampOptions(model=model, max_iter=its, stop_criteria_thr=0.0, out_dir=str(out),
                                              out_name="ex"), true_signal=beta[d.S:d.S + d.M])
                v.infere()
        except BaseException as e:  # noqa: BLE001
            errs.append((r, e))

    try:
        th = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(P)]
        [t.start() for t in th]
        [t.join(120) for t in th]
        assert not any(t.is_alive() for t in th), "loopback ranks stuck"
        assert not errs, errs
    finally:
        if old is None:
            os.environ.pop("VAMPOMI_COMM", None)
        else:
            os.environ["VAMPOMI_COMM"] = old


def _files(d):
    return sorted(f for f in os.listdir(d) if not f.startswith("."))


@pytest.mark.parametrize("model,P", [("linear", 2), ("linear", 4), ("bin_class", 2)])
def test_cli_processes_match_loopback_ranks_bytewise(tmp_path, model, P):
    N, Mt, its = 1001, 2003, 6  # Mt % P != 0: uneven shards
    Xp, yp, tp = _inputs(str(tmp_path), N, Mt, binary=model == "bin_class")
    out_p, out_l, out_1 = tmp_path / "procs", tmp_path / "loop", tmp_path / "one"
    for d in (out_p, out_l, out_1):
        d.mkdir()
    procs, logs = _launch(_cli(Xp, yp, tp, N, Mt, out_p, its, model), P, str(tmp_path), "job")
    rcs = _wait(procs, 120)
    assert rcs == [0] * P, [open(lg).read()[-2000:] for lg in logs]
    assert not os.path.exists(tmp_path / ".job.rdzv")  # rank 0 removed the rendezvous file after the join
    _loopback(N, Mt, P, Xp, yp, tp, out_l, its, model)
    files = _files(out_p)
    assert files == _files(out_l)
    assert len(files) == 2 * its + 3  # _it_K.bin, _r1_it_K.bin per iteration, three CSV files
    for f in files:
        assert (out_p / f).read_bytes() == (out_l / f).read_bytes(), f
    # against the one-process CLI: the same counts (and, linear, x1_hat within the parity bar)
    r = subprocess.run(_cli(Xp, yp, tp, N, Mt, out_1, its, model), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:]
    one = [(int(a), int(b), int(c)) for a, b, c in
           re.findall(r"it (\d+): CG iterations (\d+), onsager CG iterations (\d+)", r.stdout)]
    assert _counts(logs[0]) == one and len(one) == its
    if model == "linear":
        for it in range(1, its + 1):
            a = np.fromfile(out_p / f"ex_it_{it}.bin", dtype="<f8")
            b = np.fromfile(out_1 / f"ex_it_{it}.bin", dtype="<f8")
            assert a.shape == b.shape == (Mt,) and relerr(a, b) <= 1e-10, it


def test_cli_rank_killed_mid_run_ends_every_process(tmp_path):
    """SIGKILL one rank after the run is under way: the other process fails
    at its next collective (the peer process is gone) with a FATAL line and
    a non-zero exit status, long before VAMPOMI_COLL_TIMEOUT_S (60 s here)."""
    N, Mt, its = 2000, 4001, 100000
    Xp, yp, tp = _inputs(str(tmp_path), N, Mt)
    out = tmp_path / "out"
    out.mkdir()
    procs, logs = _launch(_cli(Xp, yp, tp, N, Mt, out, its, "linear"), 2, str(tmp_path), "kill")
    t0 = time.monotonic()
    while not _counts(logs[0]) or _counts(logs[0])[-1][0] < 3:
        assert procs[0].poll() is None and procs[1].poll() is None, [open(lg).read()[-2000:] for lg in logs]
        assert time.monotonic() - t0 < 90, "the run did not get under way"
        time.sleep(0.05)
    os.kill(procs[1].pid, signal.SIGKILL)
    t_kill = time.monotonic()
    rc0 = procs[0].wait(70)
    rc1 = procs[1].wait(10)
    waited = time.monotonic() - t_kill
    assert rc1 == -signal.SIGKILL
    assert rc0 != 0, open(logs[0]).read()[-2000:]
    assert waited < 60, waited
    txt = open(logs[0]).read()
    assert "FATAL" in txt and "exited" in txt, txt[-2000:]
