// writer.h — asynchronous per-iteration output of a VAMP run.
//
// The reference writes x1_hat/sqrt(N) and r1/sqrt(N) of every iteration
// (_it_K.bin, _r1_it_K.bin; src/vamp.cpp:235-249, src/vamp_probit.cpp:168-186,
// mpi_store_vec_to_file src/utilities.cpp:241-249) and the CSV rows
// (src/vamp.cpp:388-393) synchronously, inside the iteration.  Here the
// iteration only queues its output:
//   1. a kernel on the context's stream scales x1 and r1 by 1/sqrt(N) (IEEE
//      division, bit for bit the host's) into a device slot;
//   2. a copy stream waits for it and copies the slot into pinned host memory;
//   3. a host writer thread waits for that copy and does the pwrites (and the
//      CSV rows, in submission order).
// The context's stream never waits for the copy or the files.  Two slots: the
// submission of iteration it+2 waits (on the host) until iteration it's files
// are written.  Failures are reported by failed()/drain() and agreed over the
// ranks at the next existing collective (agree_io, vamp.cpp).
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
    ~IterWriter();  // drains every queued job, then frees its buffers

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

   private:
    struct Job {
        int slot = -1;  // -1: host-only
        std::string px, pr;
        double *hx = nullptr, *hr = nullptr;
        std::function<bool(std::string*)> fn;
    };
    void loop();
    void finish(int slot, bool ok, const std::string& msg);

    static constexpr int kSlots = 2;
    int device_ = 0;
    int64_t M_ = 0, S_ = 0;
    double sqrtN_ = 1.0;
    hipStream_t cs_ = nullptr;
    hipEvent_t ev_ready_[kSlots] = {}, ev_copied_[kSlots] = {};
    double* dbuf_[kSlots] = {};
    double* hbuf_[kSlots] = {};
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
