// options.cpp — main_meth.exe flag grammar (src/options.cpp:13-303): exact
// flag names, one value each, reference defaults (src/options.hpp:62-104),
// the reference's FATAL messages and exit-on-unknown-flag behaviour.
#include "options.h"

#include <cstdlib>
#include <cstring>
#include <functional>
#include <iostream>
#include <map>
#include <sstream>

namespace vopt {

namespace {

enum class Kind { Str, Dbl, Int, UPos, UNonNeg, DList, IList };

struct Flag {
    Kind kind;
    void* dst;
    const char* label;  // name used in the range-check message
};

}  // namespace

bool parse(int argc, char** argv, Options& o, std::string& echo) {
    const std::map<std::string, Flag> flags = {
        {"--meth-file", {Kind::Str, &o.meth_file, nullptr}},
        {"--cov-file", {Kind::Str, &o.cov_file, nullptr}},
        {"--cov-file-test", {Kind::Str, &o.cov_file_test, nullptr}},
        {"--meth-file-test", {Kind::Str, &o.meth_file_test, nullptr}},
        {"--estimate-file", {Kind::Str, &o.estimate_file, nullptr}},
        {"--r1-file", {Kind::Str, &o.r1_file, nullptr}},
        {"--cov-estimate-file", {Kind::Str, &o.cov_estimate_file, nullptr}},
        {"--run-mode", {Kind::Str, &o.run_mode, nullptr}},
        {"--phen-file", {Kind::Str, &o.phen_file, nullptr}},
        {"--true-signal-file", {Kind::Str, &o.true_signal_file, nullptr}},
        {"--phen-file-test", {Kind::Str, &o.phen_file_test, nullptr}},
        {"--vars", {Kind::DList, &o.vars, nullptr}},
        {"--probs", {Kind::DList, &o.probs, nullptr}},
        {"--test-iter-range", {Kind::IList, &o.test_iter_range, nullptr}},
        {"--verbosity", {Kind::Int, &o.verbosity, nullptr}},
        {"--learn-vars", {Kind::UNonNeg, &o.learn_vars, "--learn-vars"}},
        {"--learn-prior-delay", {Kind::UNonNeg, &o.learn_prior_delay, "--learn-prior-delay"}},
        {"--iterations", {Kind::UPos, &o.iterations, "--iterations"}},
        {"--num-mix-comp", {Kind::UPos, &o.num_mix_comp, "--num-mix-comp"}},
        {"--out-dir", {Kind::Str, &o.out_dir, nullptr}},
        {"--out-name", {Kind::Str, &o.out_name, nullptr}},
        {"--model", {Kind::Str, &o.model, nullptr}},
        {"--stop-criteria-thr", {Kind::Dbl, &o.stop_criteria_thr, nullptr}},
        {"--merge-vars-thr", {Kind::Dbl, &o.merge_vars_thr, nullptr}},
        {"--EM-err-thr", {Kind::Dbl, &o.EM_err_thr, nullptr}},
        {"--alpha-scale", {Kind::Dbl, &o.alpha_scale, nullptr}},
        {"--rho", {Kind::Dbl, &o.rho, nullptr}},
        {"--probit-var", {Kind::Dbl, &o.probit_var, nullptr}},
        {"--h2", {Kind::Dbl, &o.h2, nullptr}},
        {"--gam1", {Kind::Dbl, &o.gam1, nullptr}},
        {"--EM-max-iter", {Kind::UPos, &o.EM_max_iter, "--EM-max-iter"}},
        {"--Mt", {Kind::UPos, &o.Mt, "--Mt"}},
        {"--C", {Kind::UNonNeg, &o.C, "--C"}},
        {"--N", {Kind::UPos, &o.N, "--N"}},
        {"--N-test", {Kind::UPos, &o.N_test, "--N_test"}},
        {"--Mt-test", {Kind::UPos, &o.Mt_test, "--Mt_test"}},
        {"--CG-max-iter", {Kind::UPos, &o.CG_max_iter, "--CG-max-iter"}},
        {"--CG-err-tol", {Kind::Dbl, &o.CG_err_tol, nullptr}},
        {"--pval-method", {Kind::Str, &o.pval_method, nullptr}},
        // engine extensions
        {"--seed", {Kind::Str, nullptr, nullptr}},
        {"--batch-rhs", {Kind::Int, &o.batch_rhs, nullptr}},
    };
    std::stringstream ss;
    ss << "\nardyh command line options:\n";
    for (int i = 1; i < argc; ++i) {
        auto f = flags.find(argv[i]);
        if (f == flags.end()) {
            std::cout << "FATAL: option \"" << argv[i] << "\" unknown\n";
            return false;
        }
        if (i == argc - 1) {
            std::cout << "FATAL  : missing argument for last option \"" << argv[i]
                      << "\". Please check your input and relaunch." << std::endl;
            return false;
        }
        const std::string name = argv[i];
        const char* val = argv[++i];
        const Flag& fl = f->second;
        switch (fl.kind) {
            case Kind::Str:
                if (name == "--seed")
                    o.seed = std::strtoull(val, nullptr, 0);
                else
                    *static_cast<std::string*>(fl.dst) = val;
                ss << name << " " << val << "\n";
                break;
            case Kind::Dbl:
                *static_cast<double*>(fl.dst) = std::atof(val);
                ss << name << (name == "--probit-var" ? "" : " ") << *static_cast<double*>(fl.dst) << "\n";
                break;
            case Kind::Int:
                *static_cast<int*>(fl.dst) = std::atoi(val);
                ss << name << " " << *static_cast<int*>(fl.dst) << "\n";
                break;
            case Kind::UPos:
            case Kind::UNonNeg: {
                const int v = std::atoi(val);
                const bool pos = fl.kind == Kind::UPos;
                if (pos ? v < 1 : v < 0) {
                    std::cout << "FATAL  : option " << fl.label << " has to be a "
                              << (pos ? "strictly positive" : "non-negative") << " integer! (" << val << " was passed)"
                              << std::endl;
                    return false;
                }
                *static_cast<unsigned*>(fl.dst) = (unsigned)v;
                ss << name << " " << (unsigned)v << "\n";
                break;
            }
            case Kind::DList: {
                auto* dst = static_cast<std::vector<double>*>(fl.dst);
                dst->clear();
                std::stringstream sl(val);
                std::string item;
                while (std::getline(sl, item, ',')) dst->push_back(std::atof(item.c_str()));
                ss << name << " " << val << "\n";
                break;
            }
            case Kind::IList: {
                auto* dst = static_cast<std::vector<int>*>(fl.dst);
                std::stringstream sl(val);
                std::string item;
                size_t n = 0;
                while (std::getline(sl, item, ',')) {
                    if (n < dst->size()) (*dst)[n] = std::atoi(item.c_str());
                    ++n;
                }
                ss << name << " " << val << "\n";
                break;
            }
        }
    }
    echo = ss.str();
    if (o.meth_file.empty() && o.meth_file_test.empty()) {  // check_options (:299-303)
        std::cout << "FATAL  : no meth file provided! Please use the --meth-file option." << std::endl;
        return false;
    }
    return true;
}

}  // namespace vopt
