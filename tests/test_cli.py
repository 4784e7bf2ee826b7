"""main_meth.exe flag grammar (src/options.cpp:13-303): reference messages and
exit codes; parsing happens before any device call, so this runs without a GPU."""
import subprocess

import pytest

import vampomi_amd as va


def cli(*args):
    return subprocess.run([va.CLI_PATH, *args], capture_output=True, text=True, timeout=120)


def test_unknown_flag_is_fatal():
    r = cli("--meth-file", "x", "--pval_method", "loo")  # README spelling is not a flag
    assert r.returncode == 1 and 'FATAL: option "--pval_method" unknown' in r.stdout


def test_missing_argument():
    r = cli("--meth-file")
    assert r.returncode == 1 and 'missing argument for last option "--meth-file"' in r.stdout


@pytest.mark.parametrize("flag,val,msg", [("--N", "0", "strictly positive"), ("--iterations", "-1", "strictly positive"),
                                          ("--learn-vars", "-2", "non-negative"), ("--N-test", "0", "--N_test")])
def test_range_checks(flag, val, msg):
    r = cli("--meth-file", "x", flag, val)
    assert r.returncode == 1 and msg in r.stdout and f"({val} was passed)" in r.stdout


def test_meth_file_required():
    r = cli("--N", "10", "--Mt", "20")
    assert r.returncode == 1 and "no meth file provided" in r.stdout


def test_echo_and_unsupported_mode():
    r = cli("--meth-file", "m.bin", "--N", "10", "--Mt", "20", "--vars", "0,0.001", "--probs", "0.5,0.5",
            "--run-mode", "predict")
    assert "ardyh command line options:" in r.stdout and "--vars 0,0.001" in r.stdout
    assert "INFO   : rank    0 has 20 markers over tot Mt = 20" in r.stdout
    assert r.returncode == 1 and 'run mode "predict"' in r.stdout


def test_unknown_model_is_fatal():
    r = cli("--meth-file", "m.bin", "--N", "10", "--Mt", "20", "--model", "poisson")
    assert r.returncode == 1 and "Invalid model specification" in r.stdout
