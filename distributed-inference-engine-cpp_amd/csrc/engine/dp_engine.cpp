// Data-parallel engine: one worker, N GPUs, one process per GPU (SURVEY §2.4 "intra-worker data
// parallel", BASELINE.json config 4).
//
//   leader (rank 0, owns the HTTP worker)            followers (ranks 1..N-1)
//   ---------------------------------------          --------------------------------------
//   DpGroup::create (shm: control + input arena)     DpGroup::attach
//   communicator (RCCL unique id via the segment) <-> communicator
//   local engine: weights H2D, ncclBroadcast  ----->  local engine: weights via ncclBroadcast
//   submit(B items):                                  loop:
//     per = ceil(B / N); post descriptor  --------->    next(seq): items [r*per, (r+1)*per)
//     local shard [0, per)                              local shard (inputs read from the arena,
//     forward; ncclAllGather(logits) <------------->    H2D over this GPU's own PCIe link)
//     D2H of all N shards -> B rows, in order           forward; ncclAllGather(logits); done(seq)
//
// With CPU engines the gather runs through the segment instead (host communicator), which is what
// the multi-process CPU tests exercise.  Every rank submits exactly `per` items (the last rank pads
// with empty inputs), so all ranks run the same batch bucket and gather the same byte count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <thread>

#include "../onnx/onnx_model.h"
#include "../parallel/comm.h"
#include "../parallel/dp_group.h"
#include "engine.h"

namespace die {

namespace {

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

struct Parts {
  std::unique_ptr<DpGroup> group;
  std::unique_ptr<Communicator> comm;
  std::unique_ptr<Engine> local;
};

// Build the communicator and the local engine of this rank (collective across ranks).
void build_local(Parts& p, const std::string& path, const EngineOptions& opt) {
  EngineOptions lo = opt;
  lo.dp_world = 0;
  lo.dp_group.clear();
  // opt.max_batch is the whole DP batch (e.g. 256 over 8 GPUs): each rank runs its share
  const int world = p.group->world();
  lo.max_batch = std::max(1, (opt.max_batch + world - 1) / world);
  if (opt.device == "cpu") {
    p.comm = make_host_comm(*p.group);
    p.local = create_cpu_engine(path, lo);
  } else {
    if (hipSetDevice(opt.device_id) != hipSuccess)
      throw std::runtime_error("dp rank " + std::to_string(p.group->rank()) + ": cannot select HIP device " +
                               std::to_string(opt.device_id));
    p.comm = make_rccl_comm(*p.group);
    lo.dp_comm = p.comm.get();
    std::string why;
    p.local = create_hip_engine(path, lo, &why);
    if (!p.local) throw std::runtime_error("dp rank " + std::to_string(p.group->rank()) + ": HIP engine unavailable: " + why);
  }
  p.local->register_host_memory(p.group->arena(), p.group->arena_bytes());
}

class DpEngine : public Engine {
 public:
  DpEngine(const std::string& path, const EngineOptions& opt) : opt_(opt) {
    world_ = std::max(1, opt.dp_world);
    const size_t numel = model_input_numel(path);
    item_bytes_ = std::max(numel * sizeof(float), text_cap_for(numel, opt));
    const size_t items = static_cast<size_t>(opt.max_batch) * world_ * 3 + 64;
    const size_t arena = opt.dp_arena_mb ? opt.dp_arena_mb << 20 : item_bytes_ * items;
    parts_.group = DpGroup::create(opt.dp_group, world_, arena, 4u << 20);
    build_local(parts_, path, opt);
    if (!parts_.group->wait_joined(600000)) throw std::runtime_error("dp followers did not join");
    device_gather_ = parts_.local->device_gather();
    DpGroup* g = parts_.group.get();
    pool_ = std::make_unique<SamplePool>(
        item_bytes_ / sizeof(float), [g](size_t bytes) { return g->arena_alloc(bytes); }, [](void*) {}, 16);
    batch_ = std::make_unique<DpBatch>();
  }

  ~DpEngine() override {
    if (parts_.local) parts_.local->synchronize();
    if (parts_.group) parts_.group->stop();
    parts_.local.reset();
    parts_.comm.reset();
  }

  std::string name() const override {
    return "dp" + std::to_string(world_) + "(" + std::string(parts_.comm->backend()) + "):" + parts_.local->name();
  }
  const std::string& getModelPath() const override { return parts_.local->getModelPath(); }
  std::vector<int64_t> getInputShape() const override { return parts_.local->getInputShape(); }
  std::vector<int64_t> getOutputShape() const override { return parts_.local->getOutputShape(); }
  int max_batch() const override { return std::min(parts_.local->max_batch() * world_, kDpMaxItems); }
  SamplePool& sample_pool() override { return *pool_; }
  size_t text_capacity() const override { return std::min(parts_.local->text_capacity(), item_bytes_); }
  void wait_for_slot() override { parts_.local->wait_for_slot(); }
  void synchronize() override { parts_.local->synchronize(); }

  Json stats() const override {
    Json j = parts_.local->stats();
    j["dp_world"] = world_;
    j["dp_backend"] = parts_.comm->backend();
    j["dp_device_gather"] = device_gather_;
    j["dp_batches"] = static_cast<long long>(posted_);
    j["dp_arena_mib"] = static_cast<double>(parts_.group->arena_bytes()) / (1 << 20);
    return j;
  }

  void submit(std::vector<BatchItem> items, BatchDone done) override {
    const int B = static_cast<int>(items.size());
    if (B == 0 || B > max_batch()) {
      BatchResult r;
      r.ok = B == 0;
      if (B) r.error = "batch of " + std::to_string(B) + " exceeds dp max_batch " + std::to_string(max_batch());
      done(r);
      return;
    }
    std::lock_guard<std::mutex> g(submit_mu_);  // descriptors must be posted in submission order
    DpGroup& grp = *parts_.group;
    // items outside the arena (predict()/batchPredict()) are staged into it first
    auto temps = std::make_shared<std::vector<SampleBuffer>>();
    for (auto& it : items) {
      const void* p = it.text ? static_cast<const void*>(it.text) : static_cast<const void*>(it.input);
      if (!p || (p >= grp.arena() && p < grp.arena() + grp.arena_bytes())) continue;
      SampleBuffer sb = pool_->acquire();
      if (it.text) {
        std::memcpy(sb.data, it.text, it.text_len);
        it.text = reinterpret_cast<const char*>(sb.data);
      } else {
        const size_t n = std::min(it.len, sb.capacity);
        std::memcpy(sb.data, it.input, n * sizeof(float));
        it.input = sb.data;
        it.len = n;
      }
      temps->push_back(sb);
    }
    const int per = (B + world_ - 1) / world_;
    DpBatch& b = *batch_;
    b.B = B;
    b.per = per;
    for (int i = 0; i < B; ++i) {
      const BatchItem& it = items[i];
      DpItem d;
      if (it.text) {
        d.off = grp.offset_of(it.text);
        d.len = it.text_len;
        d.is_text = 1;
      } else {
        d.off = it.input ? grp.offset_of(it.input) : 0;
        d.len = it.input ? it.len : 0;
      }
      b.items[i] = d;
    }
    grp.post(b);
    ++posted_;
    std::vector<BatchItem> local(static_cast<size_t>(per));
    for (int j = 0; j < per && j < B; ++j) local[j] = items[j];
    const size_t out_numel = output_numel();
    parts_.local->submit(std::move(local), [this, B, per, out_numel, done, temps](BatchResult& r) {
      BatchResult o;
      o.wall_us = r.wall_us;
      o.device_us = r.device_us;
      std::vector<float> gathered;
      std::vector<int> st, nt;
      if (device_gather_) {
        o.ok = r.ok;
        o.error = r.error;
        if (r.ok) {
          o.outputs = r.outputs;  // rank-major = item order
          o.output_numel = r.output_numel;
          if (r.status) {
            st.resize(B);
            nt.resize(B);
            for (int i = 0; i < B; ++i) {
              st[i] = r.status[(i / per) * r.status_stride + i % per];
              nt[i] = r.ntok[(i / per) * r.status_stride + i % per];
            }
          }
        }
      } else {
        // host gather: every rank contributes `per` rows (zeros when its shard failed)
        std::vector<float> mine(static_cast<size_t>(per) * out_numel, 0.f);
        if (r.ok && r.outputs) std::memcpy(mine.data(), r.outputs, mine.size() * sizeof(float));
        gathered.resize(mine.size() * world_);
        try {
          parts_.group->all_gather_host(mine.data(), gathered.data(), mine.size() * sizeof(float));
          o.ok = r.ok;
          o.error = r.error;
          o.outputs = gathered.data();
          o.output_numel = out_numel;
        } catch (const std::exception& e) {
          o.ok = false;
          o.error = e.what();
        }
      }
      if (!st.empty()) {
        o.status = st.data();
        o.ntok = nt.data();
      }
      for (auto& sb : *temps) pool_->release(sb);
      done(o);
    });
  }

 private:
  EngineOptions opt_;
  int world_ = 1;
  size_t item_bytes_ = 0;
  Parts parts_;
  bool device_gather_ = false;
  std::unique_ptr<SamplePool> pool_;
  std::unique_ptr<DpBatch> batch_;
  std::mutex submit_mu_;
  long long posted_ = 0;
};

}  // namespace

std::unique_ptr<Engine> create_dp_engine(const std::string& model_path, const EngineOptions& opt) {
  return std::make_unique<DpEngine>(model_path, opt);
}

long run_dp_follower(const std::string& model_path, const EngineOptions& opt, const std::atomic<bool>* stop) {
  Parts p;
  p.group = DpGroup::attach(opt.dp_group, opt.dp_rank, 600000, stop);
  if (!p.group) return 0;
  build_local(p, model_path, opt);
  const bool device_gather = p.local->device_gather();
  const int rank = p.group->rank();
  const size_t out_numel = p.local->output_numel();
  p.group->mark_joined();
  auto b = std::make_unique<DpBatch>();
  long served = 0;
  for (uint64_t seq = 1;; ++seq) {
    if (!p.group->next(seq, *b, stop)) break;
    const int per = b->per;
    std::vector<BatchItem> items(static_cast<size_t>(per));
    for (int j = 0; j < per; ++j) {
      const int i = rank * per + j;
      if (i >= b->B) break;
      const DpItem& d = b->items[i];
      if (d.is_text) {
        items[j].text = static_cast<const char*>(p.group->at(d.off));
        items[j].text_len = d.len;
      } else if (d.len) {
        items[j].input = static_cast<const float*>(p.group->at(d.off));
        items[j].len = d.len;
      }
    }
    DpGroup* g = p.group.get();
    p.local->submit(std::move(items), [g, seq, per, out_numel, device_gather](BatchResult& r) {
      if (!device_gather) {
        std::vector<float> mine(static_cast<size_t>(per) * out_numel, 0.f);
        if (r.ok && r.outputs) std::memcpy(mine.data(), r.outputs, mine.size() * sizeof(float));
        std::vector<float> all(mine.size() * static_cast<size_t>(g->world()));
        try {
          g->all_gather_host(mine.data(), all.data(), mine.size() * sizeof(float));
        } catch (const std::exception&) {
        }
      }
      g->done(seq);
    });
    ++served;
  }
  p.local->synchronize();
  return served;
}

}  // namespace die
