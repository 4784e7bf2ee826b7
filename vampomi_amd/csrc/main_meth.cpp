// main_meth.cpp — drop-in for the reference's main_meth.exe (src/main_meth.cpp)
// in --run-mode infere (--model linear | bin_class), test and
// association_test (--pval-method loo | se): same flags, same output files.
//
// Ranks: the reference is launched with `mpirun -np P`; this binary runs one
// process per GPU, rank/size from VAMPOMI_RANK/VAMPOMI_NRANKS (or the
// torchrun variables RANK/WORLD_SIZE, LOCAL_RANK for the device).  The RCCL
// communicator id is handed from rank 0 to the others through a rendezvous
// file (VAMPOMI_RDZV, default <out-dir>/.<out-name>.rdzv).
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vampomi.h"
#include "hostio.h"
#include "options.h"

static int env_int(const char* a, const char* b, int dflt) {
    const char* v = std::getenv(a);
    if (!v && b) v = std::getenv(b);
    return v ? std::atoi(v) : dflt;
}

// rank 0 publishes the RCCL id (removing any file an earlier job left there),
// the others wait for a file of THIS job (vio::rdzv_*) up to
// VAMPOMI_RDZV_TIMEOUT_S (default 120 s, the bench's collective limit: the
// ranks of one job start together, so a longer wait means rank 0 is gone)
static bool exchange_id(const std::string& path, int rank, double not_before, unsigned char* id) {
    const std::string nonce = vio::rdzv_nonce();
    if (rank == 0) return vampomi_comm_unique_id(id) == VAMPOMI_OK && vio::rdzv_publish(path, nonce, id, VAMPOMI_UNIQUE_ID_BYTES);
    const char* e = std::getenv("VAMPOMI_RDZV_TIMEOUT_S");
    const double s = e && std::atof(e) > 0 ? std::atof(e) : 120.0;
    return vio::rdzv_fetch(path, nonce, not_before, id, VAMPOMI_UNIQUE_ID_BYTES, (int)(s * 1000.0));
}

static vampomi_ctx* g_ctx = nullptr;  // the open context: die() ends the job's communicator

static int die(const char* what) {
    std::cout << "FATAL  : " << what << ": " << vampomi_last_error() << std::endl;
    if (g_ctx) vampomi_comm_abort(g_ctx);
    return EXIT_FAILURE;
}

// a rank-local outcome every rank must share before the next collective:
// false on every rank if it is false on any (src/main_meth.cpp exits rank-locally)
static bool all_ok(vampomi_ctx* ctx, bool ok) {
    int all = 0;
    if (vampomi_all_ok(ctx, ok ? 1 : 0, &all) != VAMPOMI_OK) return false;
    return all != 0;
}

// the iteration number of an estimate / r1 file name: the text between the
// last "it_" and the last ".bin" (src/main_meth.cpp:223-226, :249-252)
static bool iteration_of(const std::string& name, std::string& it_str) {
    const size_t pos1 = name.rfind("it_") + 3, pos2 = name.rfind(".bin");
    try {
        it_str = name.substr(pos1, pos2 - pos1);
        (void)std::stoi(it_str);
    } catch (...) {
        return false;
    }
    return true;
}

// --run-mode association_test (src/main_meth.cpp:206-264)
static int association_test(vampomi_ctx* ctx, const vopt::Options& opt, int rank, int64_t M, int64_t S) {
    std::vector<double> in((size_t)std::max<int64_t>(M, 1)), pvals((size_t)std::max<int64_t>(M, 1));
    std::string it_str, out;
    if (opt.pval_method == "se") {
        if (!iteration_of(opt.r1_file, it_str)) {
            std::cout << "FATAL  : cannot parse the iteration from --r1-file \"" << opt.r1_file << "\"" << std::endl;
            return EXIT_FAILURE;
        }
        if (rank == 0) std::cout << opt.r1_file << std::endl;
        vio::read_vec(opt.r1_file, in.data(), S, M);
        if (vampomi_assoc_se(ctx, in.data(), opt.gam1, pvals.data(), VAMPOMI_MEM_HOST) != VAMPOMI_OK)
            return die("association test (se)");
        out = opt.out_dir + "/" + opt.out_name + "_it_" + it_str + "_pval_se.bin";
    } else if (opt.pval_method == "loo") {
        if (!iteration_of(opt.estimate_file, it_str)) {
            std::cout << "FATAL  : cannot parse the iteration from --estimate-file \"" << opt.estimate_file << "\""
                      << std::endl;
            return EXIT_FAILURE;
        }
        vio::read_vec(opt.estimate_file, in.data(), S, M);
        if (vampomi_assoc_loo(ctx, in.data(), pvals.data(), nullptr, VAMPOMI_MEM_HOST) != VAMPOMI_OK)
            return die("association test (loo)");
        out = opt.out_dir + "/" + opt.out_name + "_it_" + it_str + "_pval_loo.bin";
    } else {
        return 0;  // the reference computes nothing for another --pval-method
    }
    if (rank == 0) std::cout << "Storing p-values to file " + out << std::endl;
    if (!vio::store_vec(out, pvals.data(), S, M)) {
        std::cout << "FATAL  : cannot write " << out << std::endl;
        return EXIT_FAILURE;
    }
    return 0;
}

// --run-mode test (src/main_meth.cpp:112-205): R2 and squared correlation of
// A.x_est on the test set for the estimate files of iterations
// --test-iter-range, one _test.csv row each.
static int test_run(vampomi_ctx* ctx, const vopt::Options& opt, int rank, int64_t M, int64_t S) {
    const std::string csv = opt.out_dir + "/" + opt.out_name + "_test.csv";
    const bool made = rank != 0 || vio::csv_create_with_header(csv, {"iteration", "R2 test", "z correlation test"});
    if (!all_ok(ctx, made)) {
        std::cout << "FATAL  : cannot create " << csv << std::endl;
        return EXIT_FAILURE;
    }
    // file names: <prefix>it_<it>.<ext>, prefix up to the last "it", ext after
    // the FIRST '.' of the given name (:152-168)
    const std::string& est = opt.estimate_file;
    const size_t pos_dot = est.find('.');
    const std::string ext = pos_dot == std::string::npos ? std::string() : est.substr(pos_dot + 1);
    const size_t pos_it = est.rfind("it");
    if (rank == 0) std::cout << "est_file_name = " << est << std::endl;
    const int min_it = opt.test_iter_range.size() > 0 ? opt.test_iter_range[0] : 1;
    const int max_it = opt.test_iter_range.size() > 1 ? opt.test_iter_range[1] : min_it;
    if (rank == 0) std::cout << "iter range = [" << min_it << ", " << max_it << "]" << std::endl;
    std::vector<double> x((size_t)std::max<int64_t>(M, 1));
    for (int it = min_it; it <= max_it; ++it) {
        const std::string name = est.substr(0, pos_it) + "it_" + std::to_string(it) + "." + ext;
        std::fill(x.begin(), x.end(), 0.0);
        const bool ok = ext == "bin" ? vio::read_vec(name, x.data(), S, M) : vio::read_text_vec(name, x.data(), S, M);
        if (!all_ok(ctx, ok)) {
            std::cout << "FATAL  : cannot read estimate file " << name << std::endl;
            return EXIT_FAILURE;
        }
        double row[2];
        if (vampomi_test_metrics(ctx, x.data(), &row[0], &row[1], VAMPOMI_MEM_HOST) != VAMPOMI_OK)
            return die("test metrics");
        if (rank == 0) std::cout << row[0] << ", ";
        if (!all_ok(ctx, rank != 0 || vio::csv_write_row(csv, it, row, 2))) {
            std::cout << "FATAL  : cannot write " << csv << std::endl;
            return EXIT_FAILURE;
        }
    }
    if (rank == 0) std::cout << std::endl;
    return 0;
}

int main(int argc, char** argv) {
    vopt::Options opt;
    std::string echo;
    const int rank = env_int("VAMPOMI_RANK", "RANK", 0);
    const int nranks = env_int("VAMPOMI_NRANKS", "WORLD_SIZE", 1);
    if (!vopt::parse(argc, argv, opt, echo)) return EXIT_FAILURE;
    if (rank == 0) std::cout << echo << std::endl;

    int64_t M = 0, S = 0, Mm = 0;
    vampomi_divide_work(opt.Mt, nranks, rank, &M, &S, &Mm);
    std::printf("INFO   : rank %4d has %lld markers over tot Mt = %u, max Mm = %lld, starting at S = %lld\n", rank,
                (long long)M, opt.Mt, (long long)Mm, (long long)S);

    if (opt.run_mode != "infere" && opt.run_mode != "association_test" && opt.run_mode != "test") {
        std::cout << "FATAL  : run mode \"" << opt.run_mode
                  << "\" is not provided by this build (infere, test, association_test)" << std::endl;
        return EXIT_FAILURE;
    }
    if (opt.model != "linear" && opt.model != "bin_class") {  // src/vamp.cpp:98-104
        std::cout << "FATAL  : Invalid model specification! (\"" << opt.model << "\")" << std::endl;
        return EXIT_FAILURE;
    }

    unsigned char id[VAMPOMI_UNIQUE_ID_BYTES] = {0};
    std::string rdzv_path;
    // launch time (a job without a run nonce accepts only rendezvous files
    // written after it, minus a margin for ranks that start late)
    const double t_start = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    if (nranks > 1) {
        const char* rz = std::getenv("VAMPOMI_RDZV");
        const std::string path = rz ? rz : opt.out_dir + "/." + opt.out_name + ".rdzv";
        if (!exchange_id(path, rank, t_start - 120.0, id)) return die("communicator rendezvous failed");
        rdzv_path = path;
    }
    const bool test_mode = opt.run_mode == "test";  // the context holds the TEST data set (:128)
    vampomi_shard_desc d{};
    d.N = test_mode ? opt.N_test : opt.N;
    d.Mt = opt.Mt;
    d.rank = rank;
    d.nranks = nranks;
    d.device = env_int("LOCAL_RANK", nullptr, -1);
    d.comm_id = nranks > 1 ? id : nullptr;
    d.alpha_scale = opt.alpha_scale;
    vampomi_ctx* ctx = nullptr;
    if (vampomi_open(&d, &ctx) != VAMPOMI_OK) return die("cannot open the device context");
    g_ctx = ctx;
    // every rank has joined the communicator (its init is collective): the
    // rendezvous file has served and must not be read by a later job
    if (rank == 0 && !rdzv_path.empty()) vio::rdzv_remove(rdzv_path);

    // data::data: phenotype first (standardised for the linear model, raw 0/1
    // for bin_class, src/data.cpp:40-43), then the shard
    auto t0 = std::chrono::steady_clock::now();
    const int standardize = opt.model == "bin_class" ? 0 : 1;
    const std::string& phen = test_mode ? opt.phen_file_test : opt.phen_file;
    const std::string& meth = test_mode ? opt.meth_file_test : opt.meth_file;
    if (vampomi_read_phen(ctx, phen.c_str(), standardize) != VAMPOMI_OK) return die("phenotype");
    if (rank == 0) std::cout << "meth file name = " << meth << std::endl;
    if (vampomi_load_meth_file(ctx, meth.c_str()) != VAMPOMI_OK) return die("methylation data");
    // the ranks' shards load at their own pace (one rank's file may come off
    // slower storage): they meet here under a limit of their own, so the
    // first collective of the run is not the one that waits for the slowest
    // load under VAMPOMI_COLL_TIMEOUT_S
    if (nranks > 1) {
        const char* lt = std::getenv("VAMPOMI_LOAD_TIMEOUT_S");
        const double lim = lt && std::atof(lt) > 0 ? std::atof(lt) : 3600.0;
        if (vampomi_barrier_timeout(ctx, lim) != VAMPOMI_OK) return die("waiting for the other ranks' shards");
    }
    if (rank == 0)
        std::cout << "reading methylation data took "
                  << std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() << " seconds."
                  << std::endl;

    if (opt.run_mode == "association_test" || test_mode) {
        const int rc = test_mode ? test_run(ctx, opt, rank, M, S) : association_test(ctx, opt, rank, M, S);
        vampomi_barrier(ctx);
        vampomi_close(ctx);
        return rc;
    }

    std::vector<double> ts, init;
    if (!opt.true_signal_file.empty()) {  // src/main_meth.cpp:69-73
        ts.assign((size_t)M, 0.0);
        vio::read_vec(opt.true_signal_file, ts.data(), S, M);
    }
    if (!opt.estimate_file.empty()) {  // src/main_meth.cpp:75-80
        init.assign((size_t)M, 0.0);
        vio::read_vec(opt.estimate_file, init.data(), S, M);
    }

    vampomi_params p;
    vampomi_params_default(&p);
    p.gam1 = opt.gam1;
    p.h2 = opt.h2;
    p.max_iter = (int)opt.iterations;
    p.CG_max_iter = (int)opt.CG_max_iter;
    p.CG_err_tol = opt.CG_err_tol;
    p.EM_max_iter = (int)opt.EM_max_iter;
    p.EM_err_thr = opt.EM_err_thr;
    p.rho = opt.rho;
    p.learn_vars = (int)opt.learn_vars;
    p.learn_prior_delay = (int)opt.learn_prior_delay;
    p.stop_criteria_thr = opt.stop_criteria_thr;
    p.merge_vars_thr = opt.merge_vars_thr;
    if (opt.vars.size() != opt.probs.size() || opt.vars.empty() || opt.vars.size() > VAMPOMI_MAX_L) {
        std::cout << "FATAL  : --vars and --probs must have the same number (1.." << VAMPOMI_MAX_L << ") of entries"
                  << std::endl;
        return EXIT_FAILURE;
    }
    p.L = (int)opt.vars.size();
    for (int j = 0; j < p.L; ++j) {
        p.vars[j] = opt.vars[j];
        p.probs[j] = opt.probs[j];
    }
    p.seed = opt.seed;
    p.out_dir = opt.out_dir.c_str();
    p.out_name = opt.out_name.c_str();
    p.verbosity = opt.verbosity;
    p.true_signal = ts.empty() ? nullptr : ts.data();
    p.x1hat_init = init.empty() ? nullptr : init.data();
    p.batch_rhs = opt.batch_rhs;
    p.model = opt.model.c_str();

    std::vector<int> cg((size_t)p.max_iter), ons((size_t)p.max_iter);
    vampomi_result r{};
    r.cg_iters = cg.data();
    r.ons_iters = ons.data();
    // vampomi_infere step by step, so that every iteration reports its time
    // as the reference does (src/vamp.cpp:396-401, rank 0): one step is one
    // iteration, and the host waits once per iteration, at its end
    auto t1 = std::chrono::steady_clock::now();
    if (vampomi_vamp_begin(ctx, &p, &r) != VAMPOMI_OK) return die("inference");
    double total = 0.0;
    for (int stopped = 0; !stopped;) {
        const auto ts0 = std::chrono::steady_clock::now();
        if (vampomi_vamp_step(ctx, &stopped) != VAMPOMI_OK) return die("inference");
        const double it_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - ts0).count();
        total += it_s;
        const int it = r.iterations_run;
        double solve_s = 0.0;
        if (vampomi_step_phases(ctx, &solve_s, nullptr) != VAMPOMI_OK) return die("inference");
        if (rank == 0 && it >= 1)
            std::cout << "it " << it << ": CG iterations " << cg[it - 1] << ", onsager CG iterations " << ons[it - 1]
                      << "\nCG and onsager (one pass over the markers per step for both) took " << solve_s
                      << " seconds.\nTotal iteration time = " << it_s << "\nTotal computation time so far = " << total
                      << std::endl;
    }
    if (vampomi_vamp_end(ctx) != VAMPOMI_OK) return die("inference");
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    if (rank == 0)
        std::cout << "iterations run = " << r.iterations_run << ", total computation time = " << secs
                  << " s, A-passes executed = " << r.a_passes_exec << " (reference-equivalent " << r.a_passes_ref
                  << ")" << std::endl;
    vampomi_barrier(ctx);
    vampomi_close(ctx);
    return 0;
}
