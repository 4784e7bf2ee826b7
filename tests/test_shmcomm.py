"""The test-only cross-process communicator (VAMPOMI_COMM=shm,
vampomi_amd/csrc/shmcomm.cpp) on the CPU, without a device: forked ranks of
tests/native/shm_harness.cpp link the library's own object file.  Every
all-reduce is the rank-ordered sum bit for bit (also when larger than a slot:
chunked); a collective called from different sites fails on every rank; a rank
that exits makes the others fail at once instead of waiting out their limit;
a late rank is waited for at the join (which is collective, like RCCL's
communicator init).  The GPU side runs main_meth.exe as processes through it
(tests/test_gpu_cli_ranks.py)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "vampomi_amd", "build", "shmcomm.o")
SRC = os.path.join(ROOT, "tests", "native", "shm_harness.cpp")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not os.path.exists(OBJ):
        pytest.skip("vampomi_amd/build/shmcomm.o not built (make -C vampomi_amd/csrc)")
    exe = str(tmp_path_factory.mktemp("shm") / "shm_harness")
    r = subprocess.run(["g++", "-O2", "-std=c++17", SRC, OBJ, "-o", exe, "-lrt", "-pthread", "-L/opt/rocm/lib",
                        "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("cannot link the harness here: " + r.stderr[-300:])
    return exe


def _run(exe, *args, timeout=90):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    codes = [int(c) for c in re.search(r"exit codes: ([\d ]+)", r.stdout).group(1).split()]
    secs = float(re.search(r"seconds: ([\d.]+)", r.stdout).group(1))
    return codes, secs, r.stdout


@pytest.mark.parametrize("P", [2, 3, 4])
def test_rank_ordered_sums(harness, P):
    codes, _, out = _run(harness, "ok", P, 25)
    assert codes == [0] * P, out


def test_divergent_sites_fail_every_rank(harness):
    codes, secs, out = _run(harness, "mismatch", 3)
    assert all(c == 3 for c in codes), out
    assert "disagree" in out and secs < 15, out


def test_exited_rank_fails_the_others_fast(harness):
    codes, secs, out = _run(harness, "kill", 3)
    assert codes[-1] == 9 and all(c == 3 for c in codes[:-1]), out
    assert "exited" in out and secs < 15, out  # the collective limit is 20 s


def test_join_waits_for_a_late_rank(harness):
    codes, secs, out = _run(harness, "late", 3, 1500)
    assert codes == [0, 0, 0], out
    assert secs >= 1.4, out
