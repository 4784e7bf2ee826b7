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
#include <mpi.h>

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

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    if (argc < 3) return 2;
    const std::string cmd = argv[1];
    int rc = 0;
    if (cmd == "phen") {
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
