// writer.h — asynchronous per-iteration output of a VAMP run.
//
// The reference writes x1_hat/sqrt(N) and r1/sqrt(N) of every iteration
// (_it_K.bin, _r1_it_K.bin; src/vamp.cpp:235-249, src/vamp_probit.cpp:168-186,
// mpi_store_vec_to_file src/utilities.cpp:241-249) and the CSV rows
// (src/vamp.cpp:388-393) synchronously, inside the iteration.  Here the
// iteration only queues its output, two small kernels on the context's stream:
//   1. x1 and r1 scaled by 1/sqrt(N) (IEEE division, bit for bit the host's),
//      written straight into pinned, device-mapped host memory (a staging
//      slot), then
//   2. a sequence number into a mapped host word once that has landed;
// a host writer thread waits for the number and does the pwrites (and the
// CSV rows, in submission order).  No copy engine, stream event or runtime
// call stands between the iterations.  Two slots: the submission of
// iteration it+2 waits (on the host) until iteration it's files are written.
// Failures are reported by failed()/drain() and agreed over the ranks at the
// next existing collective (agree_io, vamp.cpp).  One writer per context,
// created with it.
#pragma once
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

#include "ctx.h"

class IterWriter {
   public:
    IterWriter() = default;
    IterWriter(const IterWriter&) = delete;
    IterWriter& operator=(const IterWriter&) = delete;
    ~IterWriter();  // drains every queued job, then frees its staging

    vampomi_status open(vampomi_ctx* c);
    // queues x1/sqrt(N) and r1/sqrt(N) (c->M each, device): written to the files
    // px / pr at byte c->S*8 when they are non-empty, copied to hist_x / hist_r
    // (host, may be null) otherwise or as well
    vampomi_status submit_vectors(vampomi_ctx* c, const double* x1, const double* r1, const std::string& px,
                                  const std::string& pr, double* hist_x, double* hist_r);
    // queues a host-only job (a CSV row) behind the vectors already queued;
    // fn returns false and sets its message on failure
    void submit_host(std::function<bool(std::string*)> fn);
    // true (and *msg) if any finished job failed; does not wait
    bool failed(std::string* msg);
    // waits until every queued job is done; then as failed()
    bool drain(std::string* msg);
    // a new run: forget an earlier run's failure (after drain)
    void clear_error();

   private:
    struct Job {
        int slot = -1;  // -1: host-only
        unsigned long long seq = 0;
        std::string px, pr;
        double *hx = nullptr, *hr = nullptr;
        std::function<bool(std::string*)> fn;
    };
    void loop();
    bool wait_landed(unsigned long long seq, std::string* msg);
    void finish(int slot, bool ok, const std::string& msg);

    static constexpr int kSlots = 2;
    int64_t M_ = 0, S_ = 0;
    double sqrtN_ = 1.0;
    hipStream_t st_ = nullptr;       // the context's stream (not owned)
    double* hbuf_[kSlots] = {};      // pinned, mapped: 2*M doubles each
    double* dbuf_[kSlots] = {};      // their device addresses
    unsigned long long* hflag_ = nullptr;  // mapped host word: the last landed sequence
    unsigned long long* dflag_ = nullptr;
    unsigned long long seq_ = 0;
    bool busy_[kSlots] = {};
    int next_ = 0;
    int pending_ = 0;  // queued jobs not yet finished
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Job> q_;
    bool stop_ = false, err_ = false;
    std::string msg_;
    std::thread th_;
};
