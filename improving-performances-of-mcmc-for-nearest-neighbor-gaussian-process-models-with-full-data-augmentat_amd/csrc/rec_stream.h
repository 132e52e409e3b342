// Field records streamed into a caller-owned host array while the chains run
// (nngp_records_stream; records$field[i, ] = field, update_Gaussian.R:305-311).
// nngp_record_field still writes the row into the device records; with a
// bound host array it also hands the row to this streamer, whose worker
// thread copies it out behind the main stream: device row -> pinned staging
// chunk (DMA on the worker's own stream, after an event recorded on the main
// stream right after the row was written) -> host row (memcpy on the worker,
// overlapped with the next chunk's DMA).  The end of an update call then waits
// for the last rows instead of copying every row of the call after the chains
// have finished (3 chains x 40 rows x 8 MB at n = 1e6: ~20 ms per call).
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

namespace nngp {

class RecordStreamer {
 public:
  struct Item {
    hipEvent_t ev;       // recorded on the main stream after the row was written; destroyed here
    const double* src;   // device row
    double* dst;         // host row
    size_t count;        // doubles
  };

  ~RecordStreamer() { stop(); }

  // worker + staging on `device`; false if HIP refused (then nothing runs)
  bool start(int device) {
    if (th_.joinable()) return true;
    device_ = device;
    if (hipSetDevice(device) != hipSuccess) return false;
    if (hipStreamCreateWithFlags(&st_, hipStreamNonBlocking) != hipSuccess) return false;
    for (int b = 0; b < 2; ++b) {
      if (hipHostMalloc(reinterpret_cast<void**>(&pin_[b]), kChunk * sizeof(double), hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&done_[b], hipEventDisableTiming) != hipSuccess) {
        release();
        return false;
      }
    }
    quit_ = false;
    th_ = std::thread([this] { run(); });
    return true;
  }

  void push(const Item& it) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(it);
      ++pushed_;
    }
    cv_.notify_one();
  }

  // wait until every pushed row is in its host array; the first HIP error
  // the worker met since the last drain (hipSuccess if none)
  hipError_t drain() {
    std::unique_lock<std::mutex> g(mu_);
    idle_cv_.wait(g, [this] { return completed_ == pushed_; });
    hipError_t e = err_;
    err_ = hipSuccess;
    return e;
  }

  void stop() {
    if (!th_.joinable()) return;
    drain();
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
    }
    cv_.notify_one();
    th_.join();
    release();
  }

 private:
  static constexpr size_t kChunk = size_t(1) << 19;  // doubles per staging chunk (4 MB)

  struct Chunk {
    double* dst = nullptr;
    size_t count = 0;
    int buf = 0;
    hipEvent_t item_ev = nullptr;  // set on an item's last chunk: the item is complete after it
  };

  void release() {
    for (int b = 0; b < 2; ++b) {
      if (pin_[b]) hipHostFree(pin_[b]);
      if (done_[b]) hipEventDestroy(done_[b]);
      pin_[b] = nullptr;
      done_[b] = nullptr;
    }
    if (st_) hipStreamDestroy(st_);
    st_ = nullptr;
  }

  void note(hipError_t e) {
    if (e == hipSuccess) return;
    std::lock_guard<std::mutex> g(mu_);
    if (err_ == hipSuccess) err_ = e;
  }

  // host half of a chunk: wait for its DMA, copy it out; completes its item
  void finish(Chunk& c) {
    hipError_t e = hipEventSynchronize(done_[c.buf]);
    note(e);
    if (e == hipSuccess) std::memcpy(c.dst, pin_[c.buf], c.count * sizeof(double));
    if (c.item_ev) {
      hipEventDestroy(c.item_ev);
      {
        std::lock_guard<std::mutex> g(mu_);
        ++completed_;
      }
      idle_cv_.notify_all();
    }
    c = Chunk();
  }

  void run() {
    hipSetDevice(device_);
    Chunk pending;
    bool has_pending = false;
    int buf = 0;
    for (;;) {
      Item it;
      {
        std::unique_lock<std::mutex> g(mu_);
        if (q_.empty() && has_pending) {
          g.unlock();
          finish(pending);  // nothing to overlap it with
          has_pending = false;
          continue;
        }
        cv_.wait(g, [this] { return quit_ || !q_.empty(); });
        if (q_.empty()) return;  // quit with nothing left
        it = q_.front();
        q_.pop_front();
      }
      note(hipStreamWaitEvent(st_, it.ev, 0));
      for (size_t off = 0; off < it.count || it.count == 0; off += kChunk) {
        Chunk c;
        c.count = it.count - off < kChunk ? it.count - off : kChunk;
        c.dst = it.dst + off;
        c.buf = buf;
        buf ^= 1;
        // buffer c.buf is free: its previous chunk was finished before the
        // pending one (the chunks finish in order on this thread)
        if (c.count) {
          note(hipMemcpyAsync(pin_[c.buf], it.src + off, c.count * sizeof(double), hipMemcpyDeviceToHost, st_));
        }
        note(hipEventRecord(done_[c.buf], st_));
        if (off + kChunk >= it.count) c.item_ev = it.ev;
        if (has_pending) finish(pending);  // overlaps this chunk's DMA
        pending = c;
        has_pending = true;
        if (it.count == 0) break;
      }
    }
  }

  int device_ = 0;
  hipStream_t st_ = nullptr;
  double* pin_[2] = {nullptr, nullptr};
  hipEvent_t done_[2] = {nullptr, nullptr};
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::deque<Item> q_;
  size_t pushed_ = 0, completed_ = 0;
  bool quit_ = false;
  hipError_t err_ = hipSuccess;
};

}  // namespace nngp
