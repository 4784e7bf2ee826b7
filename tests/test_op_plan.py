"""Host logic of the one-pass operator's plans (kernels.hip op_plan,
atax_team.hip team_plan) through the C ABI, no device: which kernel runs
for which N, and the invariants every team plan must keep (every team member
holds rows, teams fill the grid, one workgroup per CU at most, the member's
rows fit its loads)."""
import ctypes as C

import pytest

from vampomi_amd import _lib

lib = _lib.load()


def plan(N, M=62500, cus=256, variant=-1, K=2):
    T, S, TR, grid = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    ns = C.c_int64()
    name = C.create_string_buffer(128)
    st = lib.vampomi_dev_op_plan(N, M, cus, variant, K, C.byref(T), C.byref(S), C.byref(TR), C.byref(grid),
                                 C.byref(ns), name, 128)
    if st != 0:
        return None
    return dict(T=T.value, S=S.value, TR=TR.value, grid=grid.value, nslots=ns.value, name=name.value.decode())


def test_default_plans_of_the_baseline_shapes():
    c2, c3, c4 = plan(10000), plan(100000), plan(50000)
    # C2: a team of 2 with six loads per lane (configuration 5; 12 in round 3)
    assert c2["T"] == 2 and c2["S"] == 6 and c2["name"] == "atax_team_kernel<2, 6, 2, 3, 2, true, 2>"
    assert plan(9217)["T"] == 2 and plan(10752)["T"] == 2 and plan(10753)["T"] == 4
    assert plan(9216)["T"] == 1 and plan(9216)["name"] == "atax_team_kernel<2, 9, 1, 0, 0, false, 2>"
    assert c3["T"] == 32 and c3["S"] == 4 and c3["TR"] == 3200 and c3["nslots"] == 8
    assert c3["name"] == "atax_team_kernel<2, 4, 4, 5, 2, true, 2>"
    assert c4["T"] == 16 and c4["S"] == 4 and c4["nslots"] == 16
    assert plan(10000, variant=0)["name"] == "atax_kernel<2, 10>"


@pytest.mark.parametrize("N", [1, 2, 7, 128, 1023, 1025, 4097, 8192, 10239, 10240, 10241, 20000, 33333, 50001,
                               65536, 99999, 100000, 114688, 120000, 143360])
def test_team_plan_invariants(N):
    p = plan(N)
    assert p is not None, N
    T, S, TR, grid = p["T"], p["S"], p["TR"], p["grid"]
    assert 1 <= T <= 32 and T & (T - 1) == 0
    assert grid <= 256 and grid % T == 0 and (T == 1 or grid % (8 * T) == 0)
    assert p["nslots"] == grid // T
    if T > 1:
        assert (T - 1) * TR < N <= T * TR  # every member holds rows, the team covers N
        rows_per_step = 7 * 128
    else:
        rows_per_step = 8 * 128
    assert S * rows_per_step >= min(TR, N) and (S - 1) * rows_per_step < min(TR, N)


def test_no_plan_beyond_the_largest_team():
    # 32 members x 5 loads x 896 rows: beyond it the CG step keeps two passes
    assert plan(143360) is not None and plan(143361) is None
    assert plan(100000, K=3) is None
    assert plan(0) is None


def test_every_variant_plan_is_valid_or_refused():
    for v in [0] + [T * 10 + c for T in (1, 2, 4, 8, 16, 32) for c in range(7)]:
        for N in (1000, 10000, 50001, 100000):
            p = plan(N, variant=v)
            if p is None:
                continue
            if v == 0:
                assert p["T"] == 0
            else:
                assert p["T"] == v // 10


def mem_plan(N, Mt, nranks, rank=0, cus=256, probit=0, writer=0):
    b = C.c_int64()
    assert lib.vampomi_dev_mem_plan(N, Mt, nranks, rank, cus, probit, writer, C.byref(b)) == 0
    return b.value


HBM_BYTES = 288 * 10**9        # MI355X: 288 GB HBM3E per GPU
RUNTIME_MARGIN = 4 * 2**30     # RCCL buffers, the HIP runtime, torch's context


@pytest.mark.parametrize("n", [2, 4, 8])
def test_c3full_fits_one_mi355x_per_rank(n):
    """configs[2] (N = 100,000 x Mt = 500,000, 400 GB) sharded over n ranks:
    every rank's shard plus the engine's workspace (operator hand-off buffers,
    run state, writer) fits one GPU's 288 GB with room for RCCL and the
    runtime; the shard is most of it."""
    N, Mt = 100000, 500000
    for r in range(n):
        b = mem_plan(N, Mt, n, r, writer=1)
        M = Mt // n + (r < Mt % n)
        shard = M * N * 8
        assert shard <= b < shard * 1.02 + 2**30, (n, r, b, shard)
        assert b + RUNTIME_MARGIN < HBM_BYTES, (n, r, b / 1e9)
    assert plan(N, M=Mt // n)["T"] == 32  # every shard on the team operator


def test_bench_workloads_fit_one_mi355x():
    """The 1-GPU bench workloads: c3big (300,000 markers, 240 GB) fits; c3full
    on ONE rank (400 GB) does not, which is why it needs n >= 2."""
    assert mem_plan(100000, 300000, 1, writer=1) + RUNTIME_MARGIN < HBM_BYTES
    assert mem_plan(50000, 200000, 1, probit=1, writer=1) + RUNTIME_MARGIN < HBM_BYTES  # c4full
    assert mem_plan(100000, 500000, 1) > HBM_BYTES


def ax_plan(N, M=62500, cus=256, variant=-1, K=1):
    T, TR, S, grid, ns = (C.c_int() for _ in range(5))
    name = C.create_string_buffer(128)
    assert lib.vampomi_dev_ax_plan(N, M, cus, variant, K, C.byref(T), C.byref(TR), C.byref(S), C.byref(grid),
                                   C.byref(ns), name, 128) == 0
    return dict(T=T.value, TR=TR.value, S=S.value, grid=grid.value, nslots=ns.value, name=name.value.decode())


def test_ax_plans_of_the_baseline_shapes():
    """The team A.x plan (ax_team_kernel) where it has teams of >= 8 (C3, C4,
    C5: N above ~16k); the tile plan below, C2 included (its bits unchanged)."""
    c2, c4, c5 = ax_plan(10000, 50000), ax_plan(50000, 50000, K=4), ax_plan(100000, 62500)
    assert c2["T"] == 0 and c2["name"].startswith("ax_partial_kernel<1, 2, 8")
    assert c4["T"] == 16 and c4["S"] == 4 and c4["nslots"] == 16 and c4["name"] == "ax_team_kernel<4, 4, false>"
    assert c5["T"] == 32 and c5["TR"] == 3200 and c5["nslots"] == 8
    assert ax_plan(10000, variant=7)["T"] == 4  # the team plan on request (kbench)
    assert ax_plan(50000, variant=0)["T"] == 0


@pytest.mark.parametrize("N", [1, 2, 7, 1024, 1025, 4096, 4097, 8192, 16384, 16385, 20000, 32768, 33000, 50001,
                               65536, 99999, 100000, 114688, 131072, 131073])
@pytest.mark.parametrize("cus", [256, 304, 80])
def test_ax_team_plan_invariants(N, cus):
    """Every member holds rows, S <= 4 1024-row steps cover them, teams fill
    whole groups of 8 workgroups on the device, one slot per team."""
    p = ax_plan(N, cus=cus, variant=7)
    if p["T"] == 0:  # no team plan: rows past the largest team (<= 32, a group of 8 teams on the device) x 4 steps
        tmax = max(t for t in (1, 2, 4, 8, 16, 32) if 8 * t <= cus)
        assert N > tmax * 4096 - 127 * (tmax - 1)
        assert ax_plan(N, cus=cus)["name"].startswith("ax_partial_kernel")  # the default falls back to a tile plan
        return
    T, TR, S = p["T"], p["TR"], p["S"]
    assert (T - 1) * TR < N <= T * TR
    assert S <= 4 and S * 1024 >= min(TR, N)
    assert p["grid"] % (8 * T) == 0 and p["grid"] <= cus and p["nslots"] == p["grid"] // T


def op_lds(N, variant, K, M=62500, cus=256):
    out = (C.c_int64 * 6)()
    if lib.vampomi_dev_op_lds(N, M, cus, variant, K, out) != 0:
        return None
    return dict(zip(("head", "q", "qs", "part", "tot", "words"), list(out)))


# the operator kernels' LDS: gfx950 allows 160 KiB per workgroup; the head holds
# beta_k of the folded CG decision (k < kOpMaxK = 2) and its go word
LDS_MAX_DOUBLES = 160 * 1024 // 8
K_MAX = 2


def test_team_lds_layout_one_source_every_selectable_plan():
    """Every team plan any variant selects (configurations 0-6, T = 1..32, N
    across the plan boundaries) has one LDS layout for each system count K it
    may launch with (the head-start kernel is K = 1): the head before q, q's
    K strides, then the [2][CW][K] wave partials, then the [2][K] totals,
    disjoint, in that order, inside 160 KiB (team_plan refuses any plan whose
    layout does not fit, the launch refuses a size over the limit).  The
    layout the kernel addresses and the size the launch requests are this same
    function (atax_team.hip tm_lds)."""
    seen = 0
    for v in [T * 10 + c for T in (1, 2, 4, 8, 16, 32) for c in range(7)] + [-1]:
        for N in (1, 7, 1000, 4097, 9216, 9217, 10000, 10752, 10753, 20000, 50000, 50001, 100000, 143360):
            p = plan(N, variant=v)
            if p is None or p["T"] == 0:
                assert op_lds(N, v, 1) is None
                continue
            for K in range(1, K_MAX + 1):
                lay = op_lds(N, v, K)
                assert lay is not None, (N, v, K)
                seen += 1
                assert lay["head"] >= K_MAX + 1 and lay["q"] == lay["head"]
                assert lay["qs"] >= min(p["TR"], N) and lay["qs"] % 2 == 0  # every row of the tile; 16-byte pairs
                cw = 8 if p["T"] == 1 else 7
                assert lay["part"] == lay["q"] + K * lay["qs"]
                assert lay["tot"] == lay["part"] + 2 * cw * K
                assert lay["words"] == lay["tot"] + 2 * K <= LDS_MAX_DOUBLES, (N, v, K, lay)
            assert op_lds(N, v, K_MAX + 1) is None
    assert seen > 100
    assert op_lds(10000, 0, 1) is None  # the whole-column kernel has its own layout
