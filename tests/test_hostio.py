"""The engine's host-side file formats (vampomi_amd/csrc/hostio.cpp) against
the oracle's restatement of the reference writers/readers, byte for byte."""
import os
import subprocess

import numpy as np
import pytest

from oracle import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = tmp_path_factory.mktemp("h") / "harness"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "vampomi_amd", "csrc"),
                    os.path.join(ROOT, "tests", "hostio_harness.cpp"),
                    os.path.join(ROOT, "vampomi_amd", "csrc", "hostio.cpp"), "-o", str(exe)], check=True)
    return str(exe)


def run(h, *args):
    return subprocess.run([h, *map(str, args)], capture_output=True, text=True, check=True).stdout


def test_csv_bytes_identical_to_oracle_writer(harness, tmp_path):
    import ctypes as C

    lib = O.load()
    lib.orc_csv_header.argtypes = [C.c_char_p, C.POINTER(C.c_char_p), C.c_int]
    lib.orc_csv_row.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_int]
    hdr = ["iteration", "alpha1", "gam1", "alpha2", "gam2", "gamw"]
    rows = {1: [0.5, 1e-6, 0.9, 19.77, 2.0], 2: [0.25, 0.786, float("nan"), -1.0, 12345.678901234567],
            3: [1e5, -3.5, 0.0, 1e-300, 2.5]}  # 1e5 widens the row: later offsets shift (reference quirk)
    a, b = tmp_path / "engine.csv", tmp_path / "oracle.csv"
    run(harness, "csv", a, 0, *hdr)
    arr = (C.c_char_p * 6)(*[s.encode() for s in hdr])
    lib.orc_csv_header(str(b).encode(), arr, 6)
    for it, v in rows.items():
        run(harness, "csv", a, it, *v)
        vv = np.array(v)
        lib.orc_csv_row(str(b).encode(), it, vv.ctypes.data_as(C.c_void_p), len(v))
    ba, bb = a.read_bytes(), b.read_bytes()
    assert ba == bb
    assert ba.startswith(b"iteration, alpha1, gam1, alpha2, gam2, gamw\n") and len(ba.split(b"\n")[0]) == 43
    assert ba[44:116] == b"\0" * 72  # hole between the 44-byte header and row 1 at offset 116


def test_bin_offsets_and_no_truncation(harness, tmp_path):
    p = tmp_path / "x_it_1.bin"
    run(harness, "bin", p, 3, 1.5, 2.5)  # rank with S = 3
    run(harness, "bin", p, 0, -1, -2, -3)  # rank 0
    v = np.fromfile(p, dtype="<f8")
    assert v.tolist() == [-1, -2, -3, 1.5, 2.5]
    run(harness, "bin", p, 0, 9)  # shorter rewrite keeps the tail (CREATE|WRONLY, no truncate)
    assert np.fromfile(p, dtype="<f8").tolist() == [9, -2, -3, 1.5, 2.5]


@pytest.mark.parametrize("text", ["0 0 1.25\n1 1 -2.5\n2 2 3.0000000001\n", "0\t0\t1e-3\r\n1 1   7\n",
                                  " 0 0 5\n1 1 6\n", "a b 1 extra\nc d 2\n"])
def test_phen_reader_matches_oracle(harness, tmp_path, text):
    p = tmp_path / "y.phen"
    p.write_text(text)
    for std in (0, 1):
        out = run(harness, "phen", p, std).split()
        n = len(out)
        ref = O.read_phen(str(p), n, bool(std))
        assert np.array_equal(np.array(out, dtype=float), ref)


def test_phen_reader_na(harness, tmp_path):
    p = tmp_path / "na.phen"
    p.write_text("0 0 1\n1 1 NA\n")
    assert run(harness, "phen", p, 1).strip() == "ERR -2"


def test_fma_corrected_division_is_the_ieee_quotient(tmp_path):
    """loo_kernel divides X by sqrt(N) with a reciprocal and one fma correction
    (Markstein); it must be bit-identical to IEEE division for every N."""
    exe = tmp_path / "fastdiv"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tests", "fastdiv_check.c"),
                    "-o", str(exe), "-lm"], check=True)
    bad, tot = map(int, run(str(exe), 400000).split())
    assert tot > 5_000_000 and bad == 0


def test_pow_minus_one_is_within_one_ulp_of_the_reciprocal(tmp_path):
    """The device CG step forms beta = (1/rz_old) * rz_new where the reference
    writes pow(rz_old, -1) (src/vamp.cpp:731).  glibc's pow is not correctly
    rounded: it differs from the IEEE reciprocal on a small fraction of inputs,
    by one ulp at most (a 1e-16 relative change of the CG direction)."""
    exe = tmp_path / "powm1"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tests", "powm1_check.c"),
                    "-o", str(exe), "-lm"], check=True)
    bad, tot, maxulp = map(int, run(str(exe), 4000000).split())
    assert tot > 3_000_000 and maxulp <= 1 and bad < 0.01 * tot


def test_device_exp_is_correctly_rounded(tmp_path):
    """The probit denoiser's erfcx (src/utilities.cpp:293-363) calls exp; the
    device evaluates it as exp_cr (vampomi_amd/csrc/exp_cr.h, the same source
    compiled here): equal to the 113-bit expq rounded to double on every
    argument tried, and to glibc's exp (the reference's, the oracle's) except
    where glibc misrounds (~0.08 %, one ulp; profiles/r05_exp_cr_check.txt holds
    the 1e8-argument run)."""
    exe = tmp_path / "expcr"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tests", "exp_cr_check.c"),
                    "-o", str(exe), "-lquadmath", "-lm"], check=True)
    lines = [ln.split() for ln in run(str(exe), 300000).strip().splitlines()]
    for name, tried, cr_vs_quad, glibc_vs_quad, cr_vs_glibc, maxulp in lines[:3]:
        assert int(tried) == 300000 and int(cr_vs_quad) == 0, name
        assert int(maxulp) <= 1 and int(cr_vs_glibc) == int(glibc_vs_quad) and int(cr_vs_glibc) < 0.002 * int(tried)
    assert lines[3] == ["special", "0", "0"]


def test_cli_rendezvous_never_reads_an_earlier_jobs_file(harness, tmp_path):
    """main_meth.exe's rank rendezvous (vio::rdzv_*): a second job into the same
    out-dir must not pick up the first job's RCCL id, with a run nonce (torchrun
    / VAMPOMI_RUN_ID) or without one (file age), and rank 0 removes the file once
    the communicator is up."""
    import time

    path = str(tmp_path / ".out.rdzv")

    def env(**kw):
        e = {k: v for k, v in os.environ.items()
             if k not in ("VAMPOMI_RUN_ID", "TORCHELASTIC_RUN_ID", "MASTER_ADDR", "MASTER_PORT", "PMIX_NAMESPACE",
                          "OMPI_MCA_ess_base_jobid", "PMI_KVSNAME", "SLURM_JOB_ID", "SLURM_STEP_ID")}
        e.update(kw)
        return e

    def get(not_before, timeout_ms, **kw):
        return subprocess.run([harness, "rdzv-get", path, str(not_before), str(timeout_ms)], capture_output=True,
                              text=True, check=True, env=env(**kw)).stdout.strip()

    def pub(idtext, **kw):
        subprocess.run([harness, "rdzv-pub", path, idtext], check=True, env=env(**kw))

    # job 1 (nonce A) leaves its file behind (e.g. it crashed before clean-up)
    pub("job-one", VAMPOMI_RUN_ID="A")
    assert get(0, 2000, VAMPOMI_RUN_ID="A") == "job-one"
    # job 2 (nonce B): its ranks must wait for ITS rank 0, not read job 1's id
    assert get(0, 300, VAMPOMI_RUN_ID="B") == "TIMEOUT"
    pub("job-two", VAMPOMI_RUN_ID="B")
    assert get(0, 2000, VAMPOMI_RUN_ID="B") == "job-two"
    # torchrun's run id and the master address serve as nonces too
    pub("job-three", TORCHELASTIC_RUN_ID="t3")
    assert get(0, 300, TORCHELASTIC_RUN_ID="t2") == "TIMEOUT"
    assert get(0, 2000, TORCHELASTIC_RUN_ID="t3") == "job-three"
    pub("job-four", MASTER_ADDR="127.0.0.1", MASTER_PORT="29511")
    assert get(0, 300, MASTER_ADDR="127.0.0.1", MASTER_PORT="29512") == "TIMEOUT"
    # the MPI / PMIx job namespace and slurm's job.step too
    pub("job-five", PMIX_NAMESPACE="ns1")
    assert get(0, 300, PMIX_NAMESPACE="ns2") == "TIMEOUT"
    assert get(0, 2000, PMIX_NAMESPACE="ns1") == "job-five"
    pub("job-six", SLURM_JOB_ID="77", SLURM_STEP_ID="0")
    assert get(0, 300, SLURM_JOB_ID="77", SLURM_STEP_ID="1") == "TIMEOUT"
    # no nonce at all: a file older than the job is ignored
    pub("old")
    assert get(time.time() + 5, 300) == "TIMEOUT"
    assert get(time.time() - 60, 2000) == "old"  # (accepted once it is still there 3 s later)
    # ... and a stale file inside the time window that this job's rank 0
    # replaces while a reader looks at it: the reader takes the new id
    pub("stale")
    rd = subprocess.Popen([harness, "rdzv-get", path, str(time.time() - 60), "8000"], stdout=subprocess.PIPE,
                          text=True, env=env())
    time.sleep(1.0)
    pub("fresh")
    assert rd.communicate(timeout=30)[0].strip() == "fresh"
    # rank 0 removes the file after communicator init
    subprocess.run([harness, "rdzv-rm", path], check=True)
    assert not os.path.exists(path)
