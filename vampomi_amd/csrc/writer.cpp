// writer.cpp — see writer.h.
#include "writer.h"

#include <chrono>
#include <cmath>
#include <cstring>

#include "hostio.h"

vampomi_status IterWriter::open(vampomi_ctx* c) {
    M_ = c->M;
    S_ = c->S;
    sqrtN_ = std::sqrt((double)c->N);
    st_ = c->st;
    const size_t n = 2 * (size_t)std::max<int64_t>(M_, 1);
    for (int k = 0; k < kSlots; ++k) {
        HIPCHK(hipHostMalloc((void**)&hbuf_[k], n * 8, hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void**)&dbuf_[k], hbuf_[k], 0));
    }
    HIPCHK(hipHostMalloc((void**)&hflag_, 64, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(hflag_, 0, 64);
    HIPCHK(hipHostGetDevicePointer((void**)&dflag_, hflag_, 0));
    th_ = std::thread(&IterWriter::loop, this);
    return VAMPOMI_OK;
}

IterWriter::~IterWriter() {
    if (th_.joinable()) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();  // the loop leaves only with the queue empty
    }
    for (int k = 0; k < kSlots; ++k)
        if (hbuf_[k]) (void)hipHostFree(hbuf_[k]);
    if (hflag_) (void)hipHostFree(hflag_);
}

vampomi_status IterWriter::submit_vectors(vampomi_ctx* c, const double* x1, const double* r1, const std::string& px,
                                          const std::string& pr, double* hist_x, double* hist_r) {
    int k;
    {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !busy_[next_]; });  // its files from two iterations ago are written
        k = next_;
        next_ = (next_ + 1) % kSlots;
        busy_[k] = true;
    }
    const unsigned long long seq = ++seq_;
    hipError_t e = vk::div2_scalar(M_, x1, r1, sqrtN_, dbuf_[k], c->st);
    if (e == hipSuccess) e = vk::post_flag(dflag_, seq, c->st);
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> lk(mu_);
        busy_[k] = false;
        return fail(VAMPOMI_ERR_HIP, std::string("iteration writer: ") + hipGetErrorString(e));
    }
    Job j;
    j.slot = k;
    j.seq = seq;
    j.px = px;
    j.pr = pr;
    j.hx = hist_x;
    j.hr = hist_r;
    {
        std::lock_guard<std::mutex> lk(mu_);
        q_.push_back(std::move(j));
        ++pending_;
    }
    cv_.notify_all();
    return VAMPOMI_OK;
}

void IterWriter::submit_host(std::function<bool(std::string*)> fn) {
    Job j;
    j.fn = std::move(fn);
    {
        std::lock_guard<std::mutex> lk(mu_);
        q_.push_back(std::move(j));
        ++pending_;
    }
    cv_.notify_all();
}

void IterWriter::clear_error() {
    std::lock_guard<std::mutex> lk(mu_);
    err_ = false;
    msg_.clear();
}

bool IterWriter::failed(std::string* msg) {
    std::lock_guard<std::mutex> lk(mu_);
    if (err_ && msg) *msg = msg_;
    return err_;
}

bool IterWriter::drain(std::string* msg) {
    {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return pending_ == 0; });
    }
    return failed(msg);
}

void IterWriter::finish(int slot, bool ok, const std::string& msg) {
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (slot >= 0) busy_[slot] = false;
        --pending_;
        if (!ok && !err_) {
            err_ = true;
            msg_ = msg;
        }
    }
    cv_.notify_all();
}

// the stream has stored seq (its staging slot has landed); false if the
// stream failed first or nothing arrived within 10 minutes
bool IterWriter::wait_landed(unsigned long long seq, std::string* msg) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; ++spin) {
        if (__atomic_load_n(hflag_, __ATOMIC_ACQUIRE) >= seq) return true;
        if ((spin & 63) == 63) {
            const hipError_t e = hipStreamQuery(st_);
            if (e != hipSuccess && e != hipErrorNotReady) {
                *msg = std::string("iteration writer: ") + hipGetErrorString(e);
                return false;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::minutes(10)) {
                *msg = "iteration writer: the device did not deliver an iteration's output within 10 minutes";
                return false;
            }
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

void IterWriter::loop() {
    for (;;) {
        Job j;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) return;  // stop_ and nothing left
            j = std::move(q_.front());
            q_.pop_front();
        }
        std::string msg;
        bool ok = true;
        if (j.slot < 0) {
            ok = j.fn(&msg);
        } else if ((ok = wait_landed(j.seq, &msg))) {
            const double* hx = hbuf_[j.slot];
            const double* hr = hx + M_;
            if (j.hx) std::memcpy(j.hx, hx, (size_t)M_ * 8);
            if (j.hr) std::memcpy(j.hr, hr, (size_t)M_ * 8);
            if (!j.px.empty() && !(vio::store_vec(j.px, hx, S_, M_) && vio::store_vec(j.pr, hr, S_, M_))) {
                ok = false;
                msg = "cannot write iteration vectors " + j.px;
            }
        }
        finish(j.slot, ok, msg);
    }
}
