// Test harness for the engine's host file formats (vampomi_amd/csrc/hostio.cpp),
// built with g++ by tests/test_hostio.py (no GPU needed).
//   harness csv <path> <it> <v1> <v2> ...   (creates header "h0, h1.." when it == 0)
//   harness bin <path> <S> <v1> <v2> ...
//   harness phen <path> <standardize>       (prints the parsed values, %.17g)
//   harness rdzv-pub <path> <id-text>       (rank 0 of the CLI: publish, nonce from the environment)
//   harness rdzv-get <path> <not_before> <timeout_ms>  (another rank: prints the id text or TIMEOUT)
//   harness rdzv-rm <path>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hostio.h"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const std::string cmd = argv[1], path = argv[2];
    if (cmd == "csv") {
        const int it = std::atoi(argv[3]);
        if (it == 0) {
            std::vector<std::string> h;
            for (int i = 4; i < argc; ++i) h.push_back(argv[i]);
            return vio::csv_create_with_header(path, h) ? 0 : 1;
        }
        std::vector<double> v;
        for (int i = 4; i < argc; ++i) v.push_back(std::strtod(argv[i], nullptr));
        return vio::csv_write_row(path, it, v.data(), (int)v.size()) ? 0 : 1;
    }
    if (cmd == "bin") {
        const long long S = std::atoll(argv[3]);
        std::vector<double> v;
        for (int i = 4; i < argc; ++i) v.push_back(std::strtod(argv[i], nullptr));
        return vio::store_vec(path, v.data(), S, (long long)v.size()) ? 0 : 1;
    }
    if (cmd == "phen") {
        std::vector<double> y;
        const long long n = vio::read_phen(path, y);
        if (n < 0) {
            std::printf("ERR %lld\n", n);
            return 0;
        }
        if (std::atoi(argv[3])) vio::standardize_phen(y);
        for (double v : y) std::printf("%.17g\n", v);
        return 0;
    }
    if (cmd == "rdzv-pub") {
        char id[128] = {0};
        std::strncpy(id, argv[3], sizeof id - 1);
        return vio::rdzv_publish(path, vio::rdzv_nonce(), id, (int)sizeof id) ? 0 : 1;
    }
    if (cmd == "rdzv-get") {
        char id[128] = {0};
        if (!vio::rdzv_fetch(path, vio::rdzv_nonce(), std::strtod(argv[3], nullptr), id, (int)sizeof id,
                             std::atoi(argv[4]))) {
            std::printf("TIMEOUT\n");
            return 0;
        }
        std::printf("%s\n", id);
        return 0;
    }
    if (cmd == "rdzv-rm") {
        vio::rdzv_remove(path);
        return 0;
    }
    return 2;
}
