// options.h — main_meth.exe command line (restates src/options.hpp / options.cpp)
#pragma once
#include <string>
#include <vector>

namespace vopt {

struct Options {
    std::string meth_file, meth_file_test, phen_file, phen_file_test, true_signal_file;
    std::string estimate_file, r1_file, cov_estimate_file, cov_file, cov_file_test;
    std::string run_mode = "infere", out_dir, out_name, model = "linear", pval_method = "se";
    double stop_criteria_thr = 0.01, merge_vars_thr = 5e-1, EM_err_thr = 1e-2;
    unsigned EM_max_iter = 1, CG_max_iter = 500;
    double CG_err_tol = 1e-5;
    unsigned Mt = 0, N = 0, N_test = 0, Mt_test = 0, num_mix_comp = 10, learn_vars = 1, learn_prior_delay = 1;
    double alpha_scale = 1.0;
    unsigned redglob = 0, C = 0;
    double probit_var = 1, rho = 0.5, h2 = 0.5, gam1 = 1e-6;
    int verbosity = 0;
    unsigned iterations = 50;
    std::vector<double> vars{0, 1e-06, 6e-06, 3e-05, 2e-04, 1e-03, 6e-03, 3e-02, 2e-01, 1e+00};
    std::vector<double> probs{9.90000e-01, 5.00000e-03, 2.50000e-03, 1.25000e-03, 6.25000e-04,
                              3.12500e-04, 1.56250e-04, 7.81250e-05, 3.90625e-05, 3.90625e-05};
    std::vector<int> test_iter_range{1, 50};
    // engine extensions (not in the reference): Bernoulli seed, RHS batching
    unsigned long long seed = 0x5EED5EEDULL;
    int batch_rhs = 4;
};

// Parses argv exactly like Options::read_command_line_options + check_options:
// on a bad or unknown flag prints the reference's FATAL message to stdout and
// returns false (the CLI then exits with EXIT_FAILURE).  `echo` receives the
// "ardyh command line options" summary.
bool parse(int argc, char** argv, Options& o, std::string& echo);

}  // namespace vopt
