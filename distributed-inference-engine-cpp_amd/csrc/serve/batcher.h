// Dynamic batcher.
//
// API-compatible with the reference BatchProcessor<Req,Resp> (include/batch_processor.h:14-60):
// constructor (max_batch_size, timeout, callback), process(), start(), stop(), getMetrics() with
// the same Metrics fields.  Behavioural fixes:
//  * requests can be submitted asynchronously with a completion callback, so no caller thread is
//    blocked per in-flight request (the reference blocks an HTTP thread on future.get());
//  * the batch callback may itself be asynchronous (the HIP engine pipelines batches);
//  * two dispatch policies: GREEDY (default: work-conserving - dispatch what is queued as soon as
//    the downstream has a free slot, so batches grow exactly while the engine is busy) and DEADLINE
//    (wait up to `timeout` for a full batch).  `full_batches` counts batches of max size and
//    `timeout_batches` every smaller one (in the reference the latter is always 0);
//  * stop() fails queued requests with an error instead of destroying their promises.
#pragma once

#include <pthread.h>
#include <sys/prctl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <utility>
#include <vector>

namespace die {

enum class BatchPolicy { GREEDY, DEADLINE };

template <typename Request, typename Response>
class BatchProcessor {
 public:
  using BatchCallback = std::function<std::vector<Response>(const std::vector<Request>&)>;
  using Completion = std::function<void(Response*, std::exception_ptr)>;
  // Async batch function: must eventually call `finish(responses, error)` exactly once.
  using AsyncBatchFn =
      std::function<void(std::vector<Request>&&, std::function<void(std::vector<Response>&&, std::exception_ptr)>)>;
  // Called (on the batcher thread) before each dispatch; blocks while downstream is saturated.
  using ReadyFn = std::function<void()>;
  // Optional pacing (GREEDY): after ReadyFn, requests keep accumulating until the returned time or
  // until a full batch is queued, whichever comes first.
  using PaceFn = std::function<std::chrono::steady_clock::time_point()>;
  // Optional batch sizing: given the requests queued (capped at max_batch_size), how many to take
  // (Engine::preferred_batch); the rest stay queued, oldest first out, for the next batch.
  using SizeFn = std::function<size_t(size_t)>;

  struct Metrics {
    int64_t total_requests = 0;
    int64_t total_batches = 0;
    int64_t timeout_batches = 0;
    int64_t full_batches = 0;
    double avg_batch_size = 0.0;
  };

  BatchProcessor(size_t max_batch_size, std::chrono::milliseconds timeout, BatchCallback callback,
                 BatchPolicy policy = BatchPolicy::GREEDY)
      : max_batch_(max_batch_size ? max_batch_size : 1), timeout_(timeout), policy_(policy) {
    async_ = [cb = std::move(callback)](std::vector<Request>&& reqs,
                                        std::function<void(std::vector<Response>&&, std::exception_ptr)> finish) {
      std::vector<Response> out;
      try {
        out = cb(reqs);
      } catch (...) {
        finish(std::move(out), std::current_exception());
        return;
      }
      finish(std::move(out), nullptr);
    };
  }

  BatchProcessor(size_t max_batch_size, std::chrono::milliseconds timeout, AsyncBatchFn fn, ReadyFn ready,
                 BatchPolicy policy = BatchPolicy::GREEDY, PaceFn pace = nullptr)
      : max_batch_(max_batch_size ? max_batch_size : 1),
        timeout_(timeout),
        policy_(policy),
        async_(std::move(fn)),
        ready_(std::move(ready)),
        pace_(std::move(pace)) {}

  ~BatchProcessor() { stop(); }
  BatchProcessor(const BatchProcessor&) = delete;
  BatchProcessor& operator=(const BatchProcessor&) = delete;

  void start() {
    if (running_.exchange(true)) return;
    thread_ = std::thread([this] {
      prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // paced dispatch: wake within ~1 us, not 50 us
      pthread_setname_np(pthread_self(), "die-batcher");
      loop();
    });
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stopped_ = true;
      if (!running_.exchange(false) && !thread_.joinable()) return;
    }
    cv_.notify_all();
    if (thread_.joinable()) thread_.join();
    std::deque<Item> rest;
    {
      std::lock_guard<std::mutex> g(mu_);
      rest.swap(queue_);
    }
    auto err = std::make_exception_ptr(std::runtime_error("batch processor stopped"));
    for (auto& it : rest) it.done(nullptr, err);
  }

  // Asynchronous submission; `done` runs on the thread that finishes the batch.
  void submit(Request req, Completion done) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!stopped_) {
        queue_.push_back(Item{std::move(req), std::move(done), std::chrono::steady_clock::now()});
        total_requests_.fetch_add(1, std::memory_order_relaxed);
        done = nullptr;
      }
    }
    if (done) {  // after stop(): fail fast instead of queueing forever
      done(nullptr, std::make_exception_ptr(std::runtime_error("batch processor stopped")));
      return;
    }
    cv_.notify_one();
  }

  // Blocking submission (reference API).
  Response process(const Request& req) {
    auto pr = std::make_shared<std::promise<Response>>();
    auto fut = pr->get_future();
    submit(req, [pr](Response* r, std::exception_ptr e) {
      if (e) pr->set_exception(e);
      else pr->set_value(std::move(*r));
    });
    return fut.get();
  }

  Metrics getMetrics() const {
    std::lock_guard<std::mutex> g(metrics_mu_);
    Metrics m;
    m.total_requests = total_requests_.load();
    m.total_batches = total_batches_;
    m.timeout_batches = timeout_batches_;
    m.full_batches = full_batches_;
    m.avg_batch_size = total_batches_ ? static_cast<double>(batched_requests_) / total_batches_ : 0.0;
    return m;
  }

  // Set before start().
  void set_size_fn(SizeFn fn) { size_ = std::move(fn); }
  // Balanced batches (GREEDY): when more requests are queued than the previous batch carried, take
  // the mean of the two (rounded up), leaving the rest to lead the next batch.  In a closed loop the
  // queue at each dispatch is what the previous batch left outstanding, so consecutive batches
  // otherwise alternate large / small (sizes 26, 12, 26, ... with 50 clients), and a small batch
  // costs far more per image than the large one saves (profiles/r5_batch_curve.md).
  void set_balance(bool on) { balance_ = on; }
  // Batches dispatched per size (index = batch size, 0 unused).
  std::vector<long long> size_histogram() const {
    std::lock_guard<std::mutex> g(metrics_mu_);
    return size_hist_;
  }
  // Batches cut below the queue by balancing or the size function (and the requests left queued).
  long long trimmed_batches() const { return trimmed_batches_.load(); }
  long long trimmed_requests() const { return trimmed_requests_.load(); }

  // Total time the batcher held dispatches back for pacing.
  double paced_ms() const { return paced_ns_.load() / 1e6; }

  size_t queue_depth() const {
    std::lock_guard<std::mutex> g(mu_);
    return queue_.size();
  }
  size_t max_batch_size() const { return max_batch_; }

 private:
  struct Item {
    Request req;
    Completion done;
    std::chrono::steady_clock::time_point t;
  };

  void loop() {
    while (true) {
      std::vector<Item> batch;
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (queue_.empty()) {
          // An idle spell ends the alternation that balancing evens out: the previous batch size
          // says nothing about a burst that arrives after it.
          const auto w0 = std::chrono::steady_clock::now();
          cv_.wait(lk, [&] { return !queue_.empty() || !running_; });
          if (std::chrono::steady_clock::now() - w0 > kIdleReset) last_n_ = 0;
        }
        if (!running_) return;
        if (policy_ == BatchPolicy::DEADLINE) {
          const auto deadline = queue_.front().t + timeout_;
          cv_.wait_until(lk, deadline, [&] { return queue_.size() >= max_batch_ || !running_; });
          if (!running_) return;
        }
      }
      if (ready_) ready_();  // downstream saturated -> requests keep accumulating meanwhile
      bool full;
      {
        std::lock_guard<std::mutex> g(mu_);
        full = queue_.size() >= max_batch_;
      }
      if (pace_ && policy_ == BatchPolicy::GREEDY && !full) {
        const auto t = pace_();  // may block (e.g. until the batch in flight starts); not under mu_
        const auto w0 = std::chrono::steady_clock::now();
        if (t > w0) {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait_until(lk, t, [&] { return queue_.size() >= max_batch_ || !running_; });
          paced_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
        }
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        if (!running_) return;
        const size_t q = std::min(queue_.size(), max_batch_);
        size_t take = q;
        // Batch shaping (balanced batches, the engine's efficient sizes) only while the device is the
        // bottleneck -- a queue of at least half the max batch at dispatch: at low concurrency every
        // request cut from a batch waits a whole forward for nothing (16 client connections, shaping
        // always on: 592-856 trimmed batches and -9 % req/s, profiles/r6_batch_policy.md).  (A full
        // queue is balanced too: exempting it let 32-request batches break the 50-connection loop's
        // 24-request rhythm in the same-box A/B.)
        const bool shaping = 2 * q >= max_batch_;
        if (balance_ && shaping && policy_ == BatchPolicy::GREEDY && last_n_ > 0 && q > last_n_)
          take = (q + last_n_ + 1) / 2;
        if (size_ && shaping && take > 1) take = std::max<size_t>(1, std::min(take, size_(take)));
        if (take < q) {
          trimmed_batches_.fetch_add(1, std::memory_order_relaxed);
          trimmed_requests_.fetch_add(static_cast<long long>(q - take), std::memory_order_relaxed);
        }
        while (!queue_.empty() && batch.size() < take) {
          batch.push_back(std::move(queue_.front()));
          queue_.pop_front();
        }
      }
      if (batch.empty()) continue;
      last_n_ = batch.size();
      dispatch(std::move(batch));
    }
  }

  void dispatch(std::vector<Item>&& batch) {
    const size_t n = batch.size();
    {
      std::lock_guard<std::mutex> g(metrics_mu_);
      ++total_batches_;
      batched_requests_ += static_cast<int64_t>(n);
      if (n >= max_batch_) ++full_batches_;
      else ++timeout_batches_;
      if (size_hist_.size() <= n) size_hist_.resize(n + 1, 0);
      ++size_hist_[n];
    }
    std::vector<Request> reqs;
    reqs.reserve(n);
    auto dones = std::make_shared<std::vector<Completion>>();
    dones->reserve(n);
    for (auto& it : batch) {
      reqs.push_back(std::move(it.req));
      dones->push_back(std::move(it.done));
    }
    auto finish = [dones](std::vector<Response>&& resps, std::exception_ptr err) {
      for (size_t i = 0; i < dones->size(); ++i) {
        if (err) {
          (*dones)[i](nullptr, err);
        } else if (i < resps.size()) {
          (*dones)[i](&resps[i], nullptr);
        } else {
          (*dones)[i](nullptr, std::make_exception_ptr(std::runtime_error("No response for batched request")));
        }
      }
    };
    try {
      async_(std::move(reqs), finish);
    } catch (...) {
      finish({}, std::current_exception());
    }
  }

  size_t max_batch_;
  std::chrono::milliseconds timeout_;
  BatchPolicy policy_;
  AsyncBatchFn async_;
  ReadyFn ready_;
  PaceFn pace_;
  SizeFn size_;
  bool balance_ = false;
  size_t last_n_ = 0;  // size of the previous batch (batcher thread only)
  static constexpr std::chrono::milliseconds kIdleReset{20};  // idle wait that forgets last_n_
  std::atomic<long long> paced_ns_{0};
  std::atomic<long long> trimmed_batches_{0}, trimmed_requests_{0};
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> queue_;
  std::thread thread_;
  std::atomic<bool> running_{false};
  bool stopped_ = false;
  std::atomic<int64_t> total_requests_{0};
  mutable std::mutex metrics_mu_;
  int64_t total_batches_ = 0, timeout_batches_ = 0, full_batches_ = 0, batched_requests_ = 0;
  std::vector<long long> size_hist_;  // guarded by metrics_mu_
};

}  // namespace die
