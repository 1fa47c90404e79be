// Data-parallel engine: one logical worker, N GPUs, one process per GPU (SURVEY §2.4 "intra-worker
// data parallel", BASELINE.json config 4).  Every rank runs the same engine:
//
//   any rank r (its worker's batcher)                     leader (rank 0) dispatcher thread
//   -----------------------------------                   -------------------------------------
//   HTTP ingest (shared port, SO_REUSEPORT) -> parse       pop the oldest queued sub-batches of any
//   into the shared arena -> submit(items):                rank (up to N x local max batch), post
//     push_sub(sub-batch of arena offsets) ------------->  ONE DP batch (items + sub-batch refs)
//                                                          after pacing on the local GPU
//   shard loop: next(seq) -> items [r*per, (r+1)*per)  <-  (the leader runs shard 0 itself)
//   local forward (inputs DMA'd from the arena over this GPU's own PCIe link) ->
//   ncclAllGather(logits, decode status) -> D2H of all rows -> complete the sub-batches THIS rank
//   queued (rows [start, start + n) of the batch) -> done(seq)
//
// So HTTP/JSON ingest scales with the ranks (no single process parses every request, VERDICT r1
// "DP mode ... leader-only ingest caps scaling"), batches still form across all ranks' traffic, and
// every GPU runs the same batch bucket (each rank submits exactly `per` items) so the collectives
// match.  CPU engines gather through the segment (host communicator), which is what the multi-process
// CPU tests exercise.
#include <pthread.h>
#include <hip/hip_runtime.h>
#include <sys/prctl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>
#include <stdexcept>
#include <thread>

#include "../core/log.h"
#include "../onnx/onnx_model.h"
#include "../parallel/comm.h"
#include "../parallel/dp_group.h"
#include "../parallel/dp_layout.h"
#include "engine.h"

namespace die {

namespace {

// 64-bit hash of the whole model file: ranks must load the same bytes (plan signature).  Eight
// bytes per step (multiply + xor-shift mix) instead of byte-wise FNV: a 100-350 MB model hashes in
// tens of ms per rank (page-cache hot after the first rank), not a third of a second.
uint64_t file_hash(const std::string& path) {
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return 0;
  uint64_t h = 0xcbf29ce484222325ull, total = 0;
  std::vector<uint64_t> buf(1 << 17);  // 1 MiB
  size_t n;
  while ((n = std::fread(buf.data(), 1, buf.size() * 8, f)) > 0) {
    const size_t words = n / 8;
    for (size_t i = 0; i < words; ++i) {
      h = (h ^ buf[i]) * 0x9E3779B97F4A7C15ull;
      h ^= h >> 29;
    }
    const unsigned char* tail = reinterpret_cast<const unsigned char*>(buf.data()) + words * 8;
    for (size_t i = 0; i < n - words * 8; ++i) h = (h ^ tail[i]) * 0x100000001b3ull;
    total += n;
  }
  std::fclose(f);
  return h ^ total;
}

// What every rank's local engine must agree on before the first collective: the program (model
// bytes, precision, device type, local batch and the plan-shaping options) and the gather backend.
std::string plan_signature(const std::string& path, const EngineOptions& o, int local_max) {
  char h[17];
  std::snprintf(h, sizeof h, "%016llx", static_cast<unsigned long long>(file_hash(path)));
  return std::string(h) + "|" + (o.device == "cpu" ? "cpu" : "hip") + "|" + o.precision + "|b" +
         std::to_string(local_max) + "|" + o.dp_backend + "|dec" + std::to_string(o.device_decode) + "|pk" +
         std::to_string(o.pack_text) + "|br" + std::to_string(o.branch_streams) + "|bn" + std::to_string(o.bn_on_load) + "|fp" + std::to_string(o.fuse_pairs) + "|sp" + std::to_string(o.fuse_stem_pool) + "|gf" + std::to_string(o.fuse_gap_fc) + "|fl" + std::to_string(o.fold_layernorm) + "|le" + std::to_string(o.ln_stats_epilogue) + "|tg" + std::to_string(o.tune_in_graph) + "|to" + std::to_string(o.tune_orders) + "|tt" + std::to_string(o.tune_tail);
}

size_t model_input_numel(const std::string& path) {
  onnx::Model m = onnx::load_onnx(path);
  if (m.inputs.empty()) throw std::runtime_error("model has no inputs");
  size_t n = 1;
  for (size_t k = 1; k < m.inputs[0].dims.size(); ++k) n *= static_cast<size_t>(std::max<int64_t>(1, m.inputs[0].dims[k]));
  return n;
}

// Text capacity the HIP engine will report (kept in sync with hip_engine.hip).
size_t text_cap_for(size_t numel, const EngineOptions& opt) {
  return opt.device != "cpu" && opt.device_decode ? (numel * 24 + 4095) / 4096 * 4096 : 0;
}

// Arena sizing and back-pressure, in units of one rank's local batch (local_max_ requests):
// requests staged per rank in the arena, and requests one rank may have queued + in flight.
constexpr int kDpArenaBatches = 12;
constexpr int kDpInflightBatches = 4;

}  // namespace

// One staged request: its floats (numel x 4 B) or its input_data text.  With 4-bit packing (the
// default, core/textpack.h) a text of up to 8 characters per value fits the float-sized item (the
// bench's 4-decimal images average 7); a longer or unpackable text is parsed on the host into the
// same item (serve/worker.cpp).  Only raw (unpacked) device decode needs the worst-case text room
// of 24 bytes per value -- round 3 always reserved it: 3.45 MiB per item, 10.5 GiB of /dev/shm at
// 8 ranks x batch 256, pinned by every rank.
DpArenaPlan dp_arena_plan(size_t numel, const EngineOptions& opt, int world) {
  DpArenaPlan a;
  world = std::max(1, world);
  const int local_max = std::max(1, std::min((opt.max_batch + world - 1) / world, kDpSubMax));
  a.item_bytes = numel * sizeof(float);
  if (!opt.pack_text) a.item_bytes = std::max(a.item_bytes, text_cap_for(numel, opt));
  a.items = static_cast<size_t>(local_max) * world * kDpArenaBatches + 64;
  a.bytes = opt.dp_arena_mb ? opt.dp_arena_mb << 20 : a.item_bytes * a.items;
  return a;
}

namespace {

struct DpAbandoned : std::runtime_error {
  DpAbandoned() : std::runtime_error("data-parallel group abandoned before attach") {}
};

class DpEngine : public Engine {
 public:
  // ext_stop (followers without ingest): abandon waiting for the leader's segment once it is set.
  DpEngine(const std::string& path, const EngineOptions& opt, const std::atomic<bool>* ext_stop = nullptr)
      : opt_(opt) {
    world_ = std::max(1, opt.dp_world);
    rank_ = opt.dp_rank;
    const size_t numel = model_input_numel(path);
    const DpArenaPlan ap = dp_arena_plan(numel, opt, world_);
    item_bytes_ = ap.item_bytes;
    // opt.max_batch is the whole DP batch (e.g. 256 over 8 GPUs); each rank's share is one sub-batch
    local_max_ = std::max(1, std::min((opt.max_batch + world_ - 1) / world_, kDpSubMax));
    if (rank_ == 0) {
      // every rank stages its in-flight requests in the arena: N x (sub-batches queued + pipeline)
      group_ = DpGroup::create(opt.dp_group, world_, ap.bytes, 4u << 20);
    } else {
      group_ = DpGroup::attach(opt.dp_group, rank_, 600000, ext_stop);
      if (!group_) throw DpAbandoned();
      world_ = group_->world();
    }
    // A group of one has nothing to merge or gather: its batcher feeds a plain local engine
    // directly (same pacing, slots and pinned staging as a plain worker) instead of queueing
    // sub-batches in the shared arena for the leader's merge loop, and no communicator is formed.
    // EngineOptions::dp_force_merge keeps the N>1 path (RCCL communicator, arena staging, merge
    // loop, device gather) at world=1 for measuring and testing it.
    solo_ = world_ == 1 && !opt.dp_force_merge;
    // every rank must plan the same program before any collective sizes a buffer from its own plan
    group_->publish_signature(plan_signature(path, opt_, local_max_));
    std::string why;
    if (!group_->check_signatures(600000, &why)) {
      if (rank_ == 0) group_->stop();
      throw std::runtime_error(why);
    }
    build_local(path);
    if (rank_ == 0) {
      if (!group_->wait_joined(600000)) throw std::runtime_error("dp followers did not join");
    } else {
      group_->mark_joined();
    }
    device_gather_ = local_->device_gather();
    DpGroup* g = group_.get();
    pool_ = std::make_unique<SamplePool>(
        item_bytes_ / sizeof(float), [g](size_t bytes) { return g->arena_alloc(bytes); }, [](void*) {}, 16);
    if (rank_ == 0)
      dispatcher_ = std::thread([this] {
        prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // paced dispatch: wake within ~1 us, not 50 us
        pthread_setname_np(pthread_self(), "die-dp-lead");
        dispatch_loop();
      });
    else shard_thread_ = std::thread([this] {
        pthread_setname_np(pthread_self(), "die-dp-shard");
        follower_loop();
      });
  }

  ~DpEngine() override {
    stop_ = true;
    if (rank_ == 0 && group_) group_->stop();
    if (dispatcher_.joinable()) dispatcher_.join();
    if (shard_thread_.joinable()) shard_thread_.join();
    if (local_) local_->synchronize();
    fail_pending("data-parallel group stopped");
    local_.reset();
    comm_.reset();
  }

  std::string name() const override {
    return "dp" + std::to_string(world_) + "(" + std::string(comm_ ? comm_->backend() : "none") + "):" + local_->name();
  }
  const std::string& getModelPath() const override { return local_->getModelPath(); }
  std::vector<int64_t> getInputShape() const override { return local_->getInputShape(); }
  std::vector<int64_t> getOutputShape() const override { return local_->getOutputShape(); }
  // one submit() = one sub-batch of this rank; DP batches merge up to world x this
  int max_batch() const override { return local_max_; }
  SamplePool& sample_pool() override { return solo_ ? local_->sample_pool() : *pool_; }
  size_t text_capacity() const override {
    // a staging item holds the text 4-bit packed when the local engine unpacks on the device (two
    // characters per byte), raw otherwise; the worker checks each body against that (worker.cpp)
    return solo_ ? local_->text_capacity()
                 : std::min(local_->text_capacity(), local_->text_packing() ? 2 * item_bytes_ : item_bytes_);
  }
  bool text_packing() const override { return local_->text_packing(); }
  size_t register_host_memory(void*, size_t) override { return 0; }
  // The worker's batcher hands over whatever it has queued as soon as this returns; the leader
  // merges everything queued at dispatch time, so requests accumulate in the ring (not in the
  // batcher) while the GPU is busy.  Bounded by ring slots and by this rank's items in flight
  // (queued + in the pipeline), not by sub-batch count: tiny eager sub-batches must not starve the
  // next merge.
  std::chrono::steady_clock::time_point dispatch_not_before() override {
    return solo_ ? local_->dispatch_not_before() : std::chrono::steady_clock::now();
  }
  void wait_for_slot() override {
    if (solo_) {
      local_->wait_for_slot();
      return;
    }
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] {
      return stop_ || (pending_.size() < static_cast<size_t>(kDpSubRing - 1) &&
                       pending_items_ < static_cast<size_t>(kDpInflightBatches) * local_max_);
    });
  }
  void synchronize() override {
    if (solo_) local_->synchronize();
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait_for(lk, std::chrono::seconds(30), [&] { return stop_ || pending_.empty(); });
  }
  bool stopped() const { return group_->stopping(); }

  Json stats() const override {
    Json j = local_->stats();
    j["dp_world"] = world_;
    j["dp_rank"] = rank_;
    j["dp_backend"] = comm_ ? comm_->backend() : "none";
    j["dp_device_gather"] = device_gather_;
    j["dp_solo"] = solo_;
    j["dp_force_merge"] = opt_.dp_force_merge;
    j["dp_affinity_restores"] = rccl_affinity_restores();
    j["dp_batches"] = static_cast<long long>(batches_.load());
    j["dp_subbatches_sent"] = static_cast<long long>(subs_sent_.load());
    j["dp_subbatches_merged"] = static_cast<long long>(subs_merged_.load());
    j["dp_shard_failed_items"] = static_cast<long long>(shard_failures_.load());
    j["dp_arena_mib"] = static_cast<double>(group_->arena_bytes()) / (1 << 20);
    j["dp_pin_request_bytes"] = static_cast<long long>(pin_request_bytes_);  // this rank asked its engine to pin
    j["dp_pinned_bytes"] = static_cast<long long>(pinned_bytes_);            // the engine pinned (HIP; 0 on CPU)
    j["dp_register_ms"] = register_ms_;
    if (rank_ == 0) {
      const double nb = static_cast<double>(std::max<long long>(1, batches_.load()));
      j["dp_pop_wait_ms_per_batch"] = pop_wait_us_.load() / nb / 1000.0;
      j["dp_slot_wait_ms_per_batch"] = slot_wait_us_.load() / nb / 1000.0;
      j["dp_pace_wait_ms_per_batch"] = pace_wait_us_.load() / nb / 1000.0;
      // fairness: leader batches a sub-batch of any rank waited before riding one
      j["dp_max_sub_wait_batches"] = max_sub_wait_.load();
      j["dp_mean_sub_wait_batches"] = static_cast<double>(sub_wait_sum_.load()) / std::max<long long>(1, subs_merged_.load());
    }
    return j;
  }

  void submit(std::vector<BatchItem> items, BatchDone done) override {
    const int B = static_cast<int>(items.size());
    if (B == 0 || B > local_max_) {
      BatchResult r;
      r.ok = B == 0;
      if (B) r.error = "batch of " + std::to_string(B) + " exceeds dp sub-batch max " + std::to_string(local_max_);
      done(r);
      return;
    }
    if (solo_) {
      batches_++;
      subs_sent_++;
      local_->submit(std::move(items), std::move(done));
      return;
    }
    std::lock_guard<std::mutex> sg(submit_mu_);  // single producer of this rank's ring
    // items outside the arena (predict()/batchPredict()) are staged into it first
    Pending pd;
    pd.n = B;
    pd.done = std::move(done);
    DpSub& s = *sub_;
    s.n = B;
    for (int i = 0; i < B; ++i) {
      BatchItem it = items[i];
      const void* p = it.text ? static_cast<const void*>(it.text) : static_cast<const void*>(it.input);
      if (p && !(p >= group_->arena() && p < group_->arena() + group_->arena_bytes())) {
        SampleBuffer sb = pool_->acquire();
        if (it.text) {
          std::memcpy(sb.data, it.text, it.packed ? (it.text_len + 1) / 2 : it.text_len);
          it.text = reinterpret_cast<const char*>(sb.data);
        } else {
          const size_t n = std::min(it.len, sb.capacity);
          std::memcpy(sb.data, it.input, n * sizeof(float));
          it.input = sb.data;
          it.len = n;
        }
        pd.temps.push_back(sb);
      }
      DpItem d;
      if (it.text) {
        d.off = group_->offset_of(it.text);
        d.len = it.text_len;
        d.is_text = it.packed ? 2 : 1;
      } else {
        d.off = it.input ? group_->offset_of(it.input) : 0;
        d.len = it.input ? it.len : 0;
      }
      s.items[i] = d;
    }
    s.sub_id = ++next_sub_;
    {
      std::lock_guard<std::mutex> g(mu_);
      pending_items_ += static_cast<size_t>(B);
      pending_.emplace(s.sub_id, std::move(pd));
    }
    subs_sent_++;
    if (!group_->push_sub(s)) fail_pending("data-parallel group stopped");
  }

 private:
  struct Pending {
    int n = 0;
    BatchDone done;
    std::vector<SampleBuffer> temps;
  };

  void build_local(const std::string& path) {
    EngineOptions lo = opt_;
    lo.dp_world = 0;
    lo.dp_group.clear();
    lo.max_batch = local_max_;
    if (opt_.device == "cpu") {
      comm_ = make_host_comm(*group_);
      local_ = create_cpu_engine(path, lo);
    } else {
      if (hipSetDevice(opt_.device_id) != hipSuccess)
        throw std::runtime_error("dp rank " + std::to_string(rank_) + ": cannot select HIP device " +
                                 std::to_string(opt_.device_id));
      // dp_backend "host": the ranks gather their (small: 4 KB per image) logits and decode status
      // through the host segment instead, every rank loads the weights itself, and no RCCL
      // communicator exists.  The default "rccl" broadcasts the weights and all-gathers over xGMI.
      if (opt_.dp_backend != "rccl" && opt_.dp_backend != "host")
        throw std::runtime_error("unknown dp_backend '" + opt_.dp_backend + "' (rccl | host)");
      const bool host_comm = opt_.dp_backend == "host";
      if (host_comm) comm_ = make_host_comm(*group_);
      else if (!solo_) comm_ = make_rccl_comm(*group_);
      lo.dp_comm = solo_ || host_comm ? nullptr : comm_.get();
      device_decode_ = lo.device_decode;
      std::string why;
      local_ = create_hip_engine(path, lo, &why);
      if (!local_) throw std::runtime_error("dp rank " + std::to_string(rank_) + ": HIP engine unavailable: " + why);
    }
    if (!solo_) {
      // Every rank's engine DMAs shard items that any rank may have staged, so it pins the whole
      // shared segment: one mapping of the same physical pages per process (the segment is not
      // copied).  Timed and reported (stats dp_register_ms / dp_pinned_mib): at 8 ranks x batch 256
      // the arena is <= 2 GiB (dp_arena_plan), pinned once per rank at start-up.
      const auto t0 = std::chrono::steady_clock::now();
      pin_request_bytes_ = group_->arena_bytes();
      pinned_bytes_ = local_->register_host_memory(group_->arena(), group_->arena_bytes());
      register_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
  }

  // Leader: merge queued sub-batches into DP batches, paced on the local GPU.
  void dispatch_loop() {
    auto b = std::make_unique<DpBatch>();
    auto s = std::make_unique<DpSub>();
    const int cap = std::min(kDpMaxItems, local_max_ * world_);
    while (!stop_ && !group_->stopping()) {
      int rank = 0;
      const auto tp0 = std::chrono::steady_clock::now();
      if (!group_->pop_sub(*s, rank, 50)) continue;
      // the local pipeline has a free slot and the batch on the GPU is about to drain: everything
      // queued by then rides in this batch
      const auto tp1 = std::chrono::steady_clock::now();
      local_->wait_for_slot();
      const auto tp2 = std::chrono::steady_clock::now();
      const auto not_before = local_->dispatch_not_before();
      if (not_before > std::chrono::steady_clock::now()) std::this_thread::sleep_until(not_before);
      const auto tp3 = std::chrono::steady_clock::now();
      // where the leader's time goes between DP batches (stats: dp_*_ms_per_batch)
      pop_wait_us_ = pop_wait_us_.load() + std::chrono::duration<double, std::micro>(tp1 - tp0).count();
      slot_wait_us_ = slot_wait_us_.load() + std::chrono::duration<double, std::micro>(tp2 - tp1).count();
      pace_wait_us_ = pace_wait_us_.load() + std::chrono::duration<double, std::micro>(tp3 - tp2).count();
      b->B = 0;
      b->nsub = 0;
      // Efficient batch sizes (EngineOptions::efficient_batch, as the plain worker's batcher): the
      // local engine's start-up curve says which per-rank size to run for what is queued now; the
      // merge stops at that many items per rank (sub-batches stay whole, the rest leads the next
      // batch).  VERDICT r5 item 5: without it the DP path ran whatever was queued (21.6 images per
      // batch at world 1 against the plain worker's bucket-end 23-24, -5.7 %).
      const int queued = std::min(cap, s->n + group_->queued_items());
      const int per_q = (queued + world_ - 1) / world_;
      const int target = std::max(s->n, std::min(cap, local_->preferred_batch(per_q) * world_));
      while (true) {
        // fairness: leader batches posted between this sub-batch's queueing and the batch it rides in
        // (the next post is batch head + 1)
        const long long waited = static_cast<long long>(group_->posted()) - s->posted_at;
        if (waited > max_sub_wait_.load()) max_sub_wait_ = waited;
        sub_wait_sum_ = sub_wait_sum_.load() + waited;
        DpSubRef& ref = b->subs[b->nsub++];
        ref.rank = rank;
        ref.sub_id = s->sub_id;
        ref.start = b->B;
        ref.n = s->n;
        std::memcpy(b->items + b->B, s->items, sizeof(DpItem) * static_cast<size_t>(s->n));
        b->B += s->n;
        subs_merged_++;
        const int next = group_->peek_sub_items();
        if (next < 0 || b->B + next > target || b->nsub >= kDpMaxSubs) break;
        if (!group_->pop_sub(*s, rank, 0)) break;
      }
      b->per = (b->B + world_ - 1) / world_;
      const uint64_t seq = group_->post(*b);
      run_shard(*b, seq);
    }
  }

  // Follower: run every posted batch's shard, in order.
  void follower_loop() {
    auto b = std::make_unique<DpBatch>();
    for (uint64_t seq = 1;; ++seq) {
      if (!group_->next(seq, *b, &stop_)) break;
      run_shard(*b, seq);
    }
    stop_ = true;
    cv_.notify_all();
  }

  // This rank's shard of batch `b` (items [rank*per, rank*per + per), padded with empty items so
  // every rank runs the same bucket); on completion, every sub-batch this rank queued is answered.
  void run_shard(const DpBatch& b, uint64_t seq) {
    const int per = b.per, B = b.B;
    const DpLayout L = DpLayout::with_per(B, world_, per);
    std::vector<BatchItem> items(static_cast<size_t>(per));  // padded to `per`: every rank runs one bucket
    for (int j = 0; j < L.shard_count(rank_); ++j) {
      const DpItem& d = b.items[L.shard_begin(rank_) + j];
      if (d.is_text) {
        items[j].text = static_cast<const char*>(group_->at(d.off));
        items[j].text_len = d.len;
        items[j].packed = d.is_text == 2;
      } else if (d.len) {
        items[j].input = static_cast<const float*>(group_->at(d.off));
        items[j].len = d.len;
      }
    }
    std::vector<DpSubRef> mine;
    for (int k = 0; k < b.nsub; ++k)
      if (b.subs[k].rank == rank_) mine.push_back(b.subs[k]);
    batches_++;
    const size_t out_numel = output_numel();
    local_->submit(std::move(items), [this, seq, L, out_numel, mine](BatchResult& r) {
      std::vector<float> gathered;
      const float* rows = nullptr;
      std::vector<int> st(static_cast<size_t>(L.B), 0), nt(static_cast<size_t>(L.B), 0), rank_ok(static_cast<size_t>(world_), 0);
      bool have_status = false;
      bool ok = true;
      std::string err = r.error;
      if (device_gather_) {
        // rank-major logits: rank r's `per` rows are items [r*per, (r+1)*per), i.e. item order
        rows = r.outputs;
        if (r.rank_ok) {
          // gathered rows + shard flags (also when this rank's own shard failed: its flag is 0, so
          // dp_item_ok fails exactly its items -- the host backend's semantics)
          std::copy(r.rank_ok, r.rank_ok + world_, rank_ok.begin());
        } else {
          ok = false;  // the collectives' D2H never completed: nothing to answer from
        }
        if (ok && r.status) {
          dp_items_from_gathered(L, r.status, static_cast<size_t>(r.status_stride), st.data());
          dp_items_from_gathered(L, r.ntok, static_cast<size_t>(r.status_stride), nt.data());
          have_status = true;
        }
      } else {
        // host gather: every rank contributes `per` rows (zeros when its shard failed) and a
        // [shard ok, status x per, ntok x per] table, every batch (the flag is never optional)
        const size_t per_rows = static_cast<size_t>(L.per) * out_numel;
        std::vector<float> mine_rows(per_rows, 0.f);
        if (r.ok && r.outputs) std::memcpy(mine_rows.data(), r.outputs, per_rows * sizeof(float));
        const size_t tl = 1 + 2 * static_cast<size_t>(L.per);
        std::vector<int> mine_st(tl, 0), all_st(tl * static_cast<size_t>(world_));
        mine_st[0] = r.ok ? 1 : 0;
        if (r.ok && r.status)
          for (int j = 0; j < L.per; ++j) {
            mine_st[1 + j] = r.status[j];
            mine_st[1 + L.per + j] = r.ntok ? r.ntok[j] : 0;
          }
        gathered.resize(per_rows * static_cast<size_t>(world_));
        try {
          group_->all_gather_host(mine_rows.data(), gathered.data(), per_rows * sizeof(float));
          group_->all_gather_host(mine_st.data(), all_st.data(), tl * sizeof(int));
          rows = gathered.data();
          for (int k = 0; k < world_; ++k) rank_ok[static_cast<size_t>(k)] = all_st[static_cast<size_t>(k) * tl];
          dp_items_from_gathered(L, all_st.data() + 1, tl, st.data());
          dp_items_from_gathered(L, all_st.data() + 1 + L.per, tl, nt.data());
          have_status = device_decode_;
        } catch (const std::exception& e) {
          ok = false;
          err = e.what();
        }
      }
      if (ok) {
        // items of a failed rank's shard fail on their own; every other item is answered
        const std::vector<uint8_t> item_ok = dp_item_ok(L, rank_ok.data());
        for (int i = 0; i < L.B; ++i)
          if (!item_ok[static_cast<size_t>(i)]) {
            st[static_cast<size_t>(i)] = kItemShardFailed;
            have_status = true;
            shard_failures_++;
          }
      }
      if (!have_status) st.clear(), nt.clear();
      if (err.empty()) err = "data-parallel shard failed";
      for (const DpSubRef& ref : mine) complete(ref, ok, err, rows, out_numel, st, nt, r);
      if (rank_ != 0) group_->done(seq);
    });
  }

  void complete(const DpSubRef& ref, bool ok, const std::string& err, const float* rows, size_t out_numel,
                const std::vector<int>& st, const std::vector<int>& nt, const BatchResult& whole) {
    Pending pd;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = pending_.find(ref.sub_id);
      if (it == pending_.end()) return;
      pd = std::move(it->second);
      pending_items_ -= static_cast<size_t>(pd.n);
      pending_.erase(it);
    }
    BatchResult o;
    o.ok = ok && rows;
    o.error = ok ? std::string() : err;
    o.wall_us = whole.wall_us;
    o.device_us = whole.device_us;
    std::vector<int> s2, n2;
    if (o.ok) {
      o.outputs = rows + static_cast<size_t>(ref.start) * out_numel;
      o.output_numel = out_numel;
      if (!st.empty()) {
        s2.assign(st.begin() + ref.start, st.begin() + ref.start + ref.n);
        n2.assign(nt.begin() + ref.start, nt.begin() + ref.start + ref.n);
        o.status = s2.data();
        o.ntok = n2.data();
      }
    }
    pd.done(o);
    for (auto& sb : pd.temps) pool_->release(sb);
    cv_.notify_all();
  }

  void fail_pending(const std::string& why) {
    std::map<uint32_t, Pending> left;
    {
      std::lock_guard<std::mutex> g(mu_);
      left.swap(pending_);
      pending_items_ = 0;
    }
    for (auto& kv : left) {
      BatchResult r;
      r.ok = false;
      r.error = why;
      kv.second.done(r);
      for (auto& sb : kv.second.temps) pool_->release(sb);
    }
    cv_.notify_all();
  }

  EngineOptions opt_;
  int world_ = 1, rank_ = 0, local_max_ = 32;
  size_t item_bytes_ = 0;
  std::unique_ptr<DpGroup> group_;
  std::unique_ptr<Communicator> comm_;
  std::unique_ptr<Engine> local_;
  bool device_gather_ = false;
  bool device_decode_ = false;  // HIP ranks decode JSON text on the device (status rows to gather)
  bool solo_ = false;  // world of one: submit straight to the local engine (no merge loop)
  size_t pin_request_bytes_ = 0, pinned_bytes_ = 0;  // shared arena pinning (build_local)
  double register_ms_ = 0.0;
  std::unique_ptr<SamplePool> pool_;
  std::unique_ptr<DpSub> sub_ = std::make_unique<DpSub>();
  std::mutex submit_mu_, mu_;
  std::condition_variable cv_;
  std::map<uint32_t, Pending> pending_;
  size_t pending_items_ = 0;  // requests in this rank's queued + in-flight sub-batches (guarded by mu_)
  uint32_t next_sub_ = 0;
  std::atomic<bool> stop_{false};
  std::thread dispatcher_, shard_thread_;
  std::atomic<long long> batches_{0}, subs_sent_{0}, subs_merged_{0}, shard_failures_{0};
  std::atomic<double> pop_wait_us_{0.0}, slot_wait_us_{0.0}, pace_wait_us_{0.0};  // leader only
  std::atomic<long long> max_sub_wait_{0}, sub_wait_sum_{0};                       // leader only
};

}  // namespace

std::unique_ptr<Engine> create_dp_engine(const std::string& model_path, const EngineOptions& opt) {
  return std::make_unique<DpEngine>(model_path, opt);
}

long run_dp_follower(const std::string& model_path, const EngineOptions& opt, const std::atomic<bool>* stop) {
  // A rank without HTTP ingest: it only computes its shard of the batches other ranks queue.
  std::unique_ptr<DpEngine> e;
  try {
    e = std::make_unique<DpEngine>(model_path, opt, stop);
  } catch (const DpAbandoned&) {
    return 0;  // stopped before the leader appeared
  }
  while (!(stop && stop->load()) && !e->stopped()) std::this_thread::sleep_for(std::chrono::milliseconds(20));
  const Json s = e->stats();
  const Json* v = s.find("dp_batches");
  const long served = v ? static_cast<long>(v->as_int()) : 0;
  e.reset();
  return served;
}

}  // namespace die
