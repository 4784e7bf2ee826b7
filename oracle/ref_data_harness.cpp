// ref_data_harness.cpp — TEST INFRASTRUCTURE.  Drives the reference's own
// data-class operators, compiled from /root/reference/src/data.cpp where it
// lies (recipe: oracle/Makefile, target `ref`; binary: oracle/_ref/ref_data),
// so the CPU restatement (vamp_oracle.c) and the device path are pinned to
// the reference's code for:
//   data::compute_markers_statistics  src/data.cpp:233-283
//   data::dot_product / data::ATx      src/data.cpp:294-333
//   data::Ax                           src/data.cpp:340-373 (MPI_Allreduce on 1 rank)
//   data::read_phen                    src/data.cpp:58-110
// Only data.cpp builds here: utilities.cpp and vamp.cpp include Boost, which
// the image lacks.  data.cpp's constructor reads the matrix
// through utilities.cpp's MPI-IO helpers, so the harness sets the object's
// fields itself and calls the member functions above directly (the class's
// private section is opened for this translation unit only); the functions of
// data.cpp that need utilities.cpp are never linked in (--gc-sections).
//
//   ref_data stats <X.bin> <N> <M> <alpha_scale> <mave.out> <msig.out>
//   ref_data ax    <X.bin> <N> <M> <x.bin> <out.bin>     (statistics first, as data::data does)
//   ref_data atx   <X.bin> <N> <M> <u.bin> <out.bin>
//   ref_data phen  <phen> <N> <standardize 0|1> <out.bin>
//   ref_data time  <N> <Mt> <reps> <seed>  (bench.py's CPU leg: the reference's own Ax / ATx
//                  on a generated N x Mt matrix, OpenMP threads as set, one rank or its
//                  marker shard under `mpiexec -np P`; prints one JSON line)
#include <mpi.h>
#include <omp.h>

#include <chrono>
#include <cstdint>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>
#include <memory>
#include <new>
#include <string>
#include <vector>

#define private public
#include "data.hpp"
#undef private

static std::vector<double> read_bin(const char* path, size_t n) {
    std::vector<double> v(n, 0.0);
    FILE* f = std::fopen(path, "rb");
    if (!f || std::fread(v.data(), 8, n, f) != n) {
        std::fprintf(stderr, "cannot read %zu doubles from %s\n", n, path);
        std::exit(3);
    }
    std::fclose(f);
    return v;
}

static void write_bin(const char* path, const double* v, size_t n) {
    FILE* f = std::fopen(path, "wb");
    if (!f || std::fwrite(v, 8, n, f) != n) std::exit(4);
    std::fclose(f);
}

// a data object with the fields data::data would set (src/data.cpp:23-46)
struct Obj {
    alignas(data) unsigned char raw[sizeof(data)];
    data* d;
    Obj(int N, int M, double alpha_scale) {
        std::memset(raw, 0, sizeof raw);
        d = reinterpret_cast<data*>(raw);
        new (&d->phenfp) std::string();
        new (&d->methfp) std::string();
        new (&d->data_class) std::string();
        new (&d->phen_data) std::vector<double>();
        d->N = N;
        d->M = M;
        d->Mt = M;
        d->S = 0;
        d->rank = 0;
        d->nonas = N;  // read_phen asserts N rows (:85)
        d->alpha_scale = alpha_scale;
        d->mave = (double*)_mm_malloc(size_t(M) * sizeof(double), 32);
        d->msig = (double*)_mm_malloc(size_t(M) * sizeof(double), 32);
    }
};

static uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Times the reference's Ax and ATx (src/data.cpp:294-373) as the reference
// runs them: under `mpiexec -np P` every rank owns its divide_work share of
// the Mt markers (src/utilities.cpp:207-239: the first Mt % P ranks one
// more), generates only those columns of an N x Mt marker-major matrix of
// uniform values (timing only; the values do not matter, and they are the
// same for every P: indexed by the GLOBAL marker), and runs data::Ax -- its
// per-marker OpenMP loop and its MPI_Allreduce of the N-vector (:349-367) --
// and data::ATx on its shard.  Each call starts after an MPI_Barrier; its
// time is the slowest rank's (MPI_MAX), i.e. the job's.  Rank 0 prints one
// JSON line: np, OpenMP threads per rank, ms per call.
static int time_ops(int N, int Mt, int reps, uint64_t seed) {
    int rank = 0, np = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &np);
    const int M = Mt / np + (rank < Mt % np ? 1 : 0);
    const int S = rank * (Mt / np) + (rank < Mt % np ? rank : Mt % np);
    const size_t n = size_t(N) * size_t(M > 0 ? M : 1);
    double* X = (double*)_mm_malloc(n * sizeof(double), 64);  // as data::read_methylation_data (:129)
    if (!X) return 5;
#pragma omp parallel for schedule(static)
    for (long long m = 0; m < M; ++m)
        for (int j = 0; j < N; ++j)
            X[size_t(m) * N + j] =
                double(splitmix(seed ^ (size_t(S + m) * N + j)) >> 11) * 0x1.0p-53 * 3.4 - 1.7;
    Obj o(N, M > 0 ? M : 1, 1.0);
    o.d->M = M;
    o.d->Mt = Mt;
    o.d->S = S;
    o.d->rank = rank;
    o.d->meth_data = X;
    o.d->compute_markers_statistics();
    std::vector<double> x(M > 0 ? M : 1), u(N);
    for (int i = 0; i < M; ++i) x[i] = double(splitmix(seed + 1 + S + i) >> 11) * 0x1.0p-53 - 0.5;
    for (int j = 0; j < N; ++j) u[j] = double(splitmix(seed + 7 + j) >> 11) * 0x1.0p-53 - 0.5;
    using clk = std::chrono::steady_clock;
    double ax = 0, atx = 0, chk = 0;
    for (int r = 0; r < reps; ++r) {
        MPI_Barrier(MPI_COMM_WORLD);
        auto t0 = clk::now();
        std::vector<double> a = o.d->Ax(x.data());
        auto t1 = clk::now();
        MPI_Barrier(MPI_COMM_WORLD);
        auto t2 = clk::now();
        std::vector<double> b = o.d->ATx(u.data());
        auto t3 = clk::now();
        double t[2] = {std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t3 - t2).count()};
        MPI_Allreduce(MPI_IN_PLACE, t, 2, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        ax += t[0];
        atx += t[1];
        chk += a[0] + (M > 0 ? b[0] : 0.0);
    }
    if (rank == 0)
        std::printf("{\"N\": %d, \"M\": %d, \"reps\": %d, \"np\": %d, \"threads\": %d, \"ax_ms\": %.3f, "
                    "\"atx_ms\": %.3f, \"check\": %.6g}\n",
                    N, Mt, reps, np, omp_get_max_threads(), ax / reps * 1e3, atx / reps * 1e3, chk);
    _mm_free(X);
    return 0;
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    if (argc < 3) return 2;
    const std::string cmd = argv[1];
    int rc = 0;
    if (cmd == "time") {
        if (argc < 6) return 2;
        rc = time_ops(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::strtoull(argv[5], nullptr, 10));
    } else if (cmd == "phen") {
        const int N = std::atoi(argv[3]);
        Obj o(N, 1, 1.0);
        o.d->phenfp = argv[2];
        o.d->read_phen(std::atoi(argv[4]) != 0);
        write_bin(argv[5], o.d->phen_data.data(), o.d->phen_data.size());
    } else {
        const int N = std::atoi(argv[3]), M = std::atoi(argv[4]);
        std::vector<double> X = read_bin(argv[2], size_t(N) * size_t(M));
        Obj o(N, M, cmd == "stats" ? std::atof(argv[5]) : 1.0);
        o.d->meth_data = X.data();
        o.d->compute_markers_statistics();
        if (cmd == "stats") {
            write_bin(argv[6], o.d->mave, size_t(M));
            write_bin(argv[7], o.d->msig, size_t(M));
        } else if (cmd == "ax") {
            std::vector<double> x = read_bin(argv[5], size_t(M));
            std::vector<double> out = o.d->Ax(x.data());
            write_bin(argv[6], out.data(), out.size());
        } else if (cmd == "atx") {
            std::vector<double> u = read_bin(argv[5], size_t(N));
            std::vector<double> out = o.d->ATx(u.data());
            write_bin(argv[6], out.data(), out.size());
        } else {
            rc = 2;
        }
    }
    MPI_Finalize();
    return rc;
}
