"""The C ABI: libvampomi loads and exports every symbol include/vampomi.h
declares, the ctypes mirror has the header's struct layout, host-only entry
points behave, and no entry point aborts the process without a GPU."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import vampomi_amd as va
from vampomi_amd import _lib
from oracle import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "vampomi.h")


def declared():
    txt = open(HDR).read()
    return set(re.findall(r"^\s*(?:vampomi_status|void|int|const char\s*\*)\s+(vampomi_\w+)\s*\(", txt, re.M))


def test_every_declared_symbol_is_exported_and_bound():
    names = declared()
    assert len(names) >= 30
    lib = C.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert names == set(_lib.SIGNATURES), names ^ set(_lib.SIGNATURES)
    assert va.load().vampomi_abi_version() == 3


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "vampomi.h"
#define P(T, f) printf(#T "." #f " %zu\n", offsetof(T, f))
int main(void) {
  printf("vampomi_shard_desc %zu\nvampomi_params %zu\nvampomi_result %zu\nvampomi_stats %zu\n",
         sizeof(vampomi_shard_desc), sizeof(vampomi_params), sizeof(vampomi_result), sizeof(vampomi_stats));
  P(vampomi_params, seed); P(vampomi_params, out_dir); P(vampomi_params, batch_rhs); P(vampomi_params, model);
  P(vampomi_result, probs_final); P(vampomi_result, L_final); P(vampomi_result, a_passes_exec);
  P(vampomi_shard_desc, comm_id); P(vampomi_shard_desc, alpha_scale); P(vampomi_stats, host_syncs);
  return 0; }''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                       check=True).stdout.splitlines())
    assert int(got["vampomi_shard_desc"]) == C.sizeof(_lib.ShardDesc)
    assert int(got["vampomi_params"]) == C.sizeof(_lib.Params)
    assert int(got["vampomi_result"]) == C.sizeof(_lib.Result)
    assert int(got["vampomi_stats"]) == C.sizeof(_lib.Stats)
    for key, val in got.items():
        if "." in key:
            t, f = key.split(".")
            cls = {"vampomi_params": _lib.Params, "vampomi_result": _lib.Result, "vampomi_shard_desc": _lib.ShardDesc,
                   "vampomi_stats": _lib.Stats}[t]
            assert getattr(cls, f).offset == int(val), key


def test_params_default_is_the_reference_cli_default():
    # src/options.hpp:62-104 (the code defaults, not the README table)
    p = va.VampOptions().to_struct()
    assert (p.gam1, p.h2, p.max_iter, p.CG_max_iter, p.CG_err_tol) == (1e-6, 0.5, 50, 500, 1e-5)
    assert (p.EM_max_iter, p.EM_err_thr, p.rho, p.learn_vars, p.learn_prior_delay) == (1, 1e-2, 0.5, 1, 1)
    assert (p.stop_criteria_thr, p.merge_vars_thr, p.L) == (0.01, 0.5, 10)
    assert list(p.vars[:10]) == [0, 1e-06, 6e-06, 3e-05, 2e-04, 1e-03, 6e-03, 3e-02, 2e-01, 1e+00]
    assert p.probs[0] == 0.99 and p.probs[9] == 3.90625e-05 and p.batch_rhs == 4
    q = _lib.Params()
    va.load().vampomi_params_default(C.byref(q))
    assert q.model == b"linear" and q.max_iter == 50


@pytest.mark.parametrize("Mt,P", [(2000, 1), (2000, 3), (500000, 8), (17, 4)])
def test_divide_work_matches_oracle(Mt, P):
    for r in range(P):
        assert va.divide_work(Mt, P, r) == O.divide_work(Mt, P, r)


def test_open_without_device_is_an_error_status_not_an_abort():
    code = ("import vampomi_amd as va\n"
            "try:\n    va.Data(100, 200)\n    print('opened')\n"
            "except va.VampomiError as e:\n    print('status', e.status)\n")
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() in ("opened", "status 2")


def test_bad_arguments_are_rejected_before_any_device_call():
    lib = va.load()
    h = C.c_void_p()
    d = _lib.ShardDesc(N=1, Mt=10, rank=0, nranks=1, device=-1, comm_id=None, alpha_scale=1.0)
    assert lib.vampomi_open(C.byref(d), C.byref(h)) == 1  # ERR_ARG: N < 2
    d = _lib.ShardDesc(N=10, Mt=10, rank=0, nranks=2, device=-1, comm_id=None, alpha_scale=1.0)
    assert lib.vampomi_open(C.byref(d), C.byref(h)) == 1  # nranks > 1 without a communicator id
    assert b"communicator" in lib.vampomi_last_error()
    assert lib.vampomi_ax(None, None, None, 0) == 1
