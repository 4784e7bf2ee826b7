// writer.cpp — see writer.h.
#include "writer.h"

#include <cmath>
#include <cstring>

#include "hostio.h"

vampomi_status IterWriter::open(vampomi_ctx* c) {
    device_ = c->device;
    M_ = c->M;
    S_ = c->S;
    sqrtN_ = std::sqrt((double)c->N);
    const size_t n = 2 * (size_t)std::max<int64_t>(M_, 1);
    HIPCHK(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking));
    for (int k = 0; k < kSlots; ++k) {
        STCHK(dev_alloc(&dbuf_[k], n));
        HIPCHK(hipHostMalloc((void**)&hbuf_[k], n * 8, hipHostMallocDefault));
        HIPCHK(hipEventCreateWithFlags(&ev_ready_[k], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_copied_[k], hipEventDisableTiming));
    }
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
    for (int k = 0; k < kSlots; ++k) {
        if (ev_ready_[k]) (void)hipEventDestroy(ev_ready_[k]);
        if (ev_copied_[k]) (void)hipEventDestroy(ev_copied_[k]);
        if (hbuf_[k]) (void)hipHostFree(hbuf_[k]);
        dev_free(dbuf_[k]);
    }
    if (cs_) (void)hipStreamDestroy(cs_);
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
    auto undo = [&](vampomi_status s) {
        std::lock_guard<std::mutex> lk(mu_);
        busy_[k] = false;
        return s;
    };
    const size_t bytes = 2 * (size_t)M_ * 8;
    hipError_t e = vk::div2_scalar(M_, x1, r1, sqrtN_, dbuf_[k], c->st);
    if (e == hipSuccess) e = hipEventRecord(ev_ready_[k], c->st);
    if (e == hipSuccess) e = hipStreamWaitEvent(cs_, ev_ready_[k], 0);
    if (e == hipSuccess && bytes) e = hipMemcpyAsync(hbuf_[k], dbuf_[k], bytes, hipMemcpyDeviceToHost, cs_);
    if (e == hipSuccess) e = hipEventRecord(ev_copied_[k], cs_);
    if (e != hipSuccess) return undo(fail(VAMPOMI_ERR_HIP, std::string("iteration writer: ") + hipGetErrorString(e)));
    Job j;
    j.slot = k;
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

void IterWriter::loop() {
    (void)hipSetDevice(device_);
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
        } else {
            const hipError_t e = hipEventSynchronize(ev_copied_[j.slot]);
            if (e != hipSuccess) {
                ok = false;
                msg = std::string("iteration writer: ") + hipGetErrorString(e);
            } else {
                const double* hx = hbuf_[j.slot];
                const double* hr = hx + M_;
                if (j.hx) std::memcpy(j.hx, hx, (size_t)M_ * 8);
                if (j.hr) std::memcpy(j.hr, hr, (size_t)M_ * 8);
                if (!j.px.empty() && !(vio::store_vec(j.px, hx, S_, M_) && vio::store_vec(j.pr, hr, S_, M_))) {
                    ok = false;
                    msg = "cannot write iteration vectors " + j.px;
                }
            }
        }
        finish(j.slot, ok, msg);
    }
}
