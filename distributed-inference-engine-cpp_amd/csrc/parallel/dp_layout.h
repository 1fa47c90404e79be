// Row bookkeeping of one data-parallel batch, as pure functions (no engine, no group), so the
// mapping every rank applies to gathered rows is unit-tested on the CPU for any world size
// (tests/test_dp.py::test_dp_layout_*, through capi die_dp_layout_*).
//
// A DP batch holds B items in the leader's merge order.  Every rank runs the same batch bucket so
// the collectives match: per = ceil(B / world) items each, rank r computes items
// [r * per, min(B, (r + 1) * per)) and pads its shard to `per`.  Collectives concatenate the
// ranks' blocks rank-major: rank r's block starts at r * stride in a gathered buffer (stride =
// per rows for logits, the engine's status-table length for decode status).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace die {

struct DpLayout {
  int B = 0;      // items in the whole batch
  int world = 1;  // ranks
  int per = 0;    // items per rank (each rank's shard is padded to this)

  static DpLayout make(int B, int world) {
    DpLayout l;
    l.B = std::max(0, B);
    l.world = std::max(1, world);
    l.per = (l.B + l.world - 1) / l.world;
    return l;
  }
  static DpLayout with_per(int B, int world, int per) {
    DpLayout l = make(B, world);
    l.per = per;
    return l;
  }
  // the rank that computes item i
  int rank_of(int i) const { return per > 0 ? i / per : 0; }
  int shard_begin(int r) const { return std::min(B, r * per); }
  // real (unpadded) items of rank r's shard
  int shard_count(int r) const { return std::max(0, std::min(B, (r + 1) * per) - shard_begin(r)); }
  // item i's entry in a rank-major gathered buffer whose rank blocks are `stride` entries apart
  size_t gathered_index(int i, size_t stride) const {
    return static_cast<size_t>(rank_of(i)) * stride + static_cast<size_t>(i - rank_of(i) * per);
  }
};

// out[i] = gathered[L.gathered_index(i, stride)] for every item i (decode status, token counts).
template <typename T>
void dp_items_from_gathered(const DpLayout& L, const T* gathered, size_t stride, T* out) {
  for (int i = 0; i < L.B; ++i) out[i] = gathered[L.gathered_index(i, stride)];
}

// Rows of item i, i in [0, B), from a rank-major row gather (rows_per_rank rows per rank block,
// row_len values each): copies into `out` in item order.
template <typename T>
void dp_rows_from_gathered(const DpLayout& L, const T* gathered, size_t rows_per_rank, size_t row_len, T* out) {
  for (int i = 0; i < L.B; ++i) {
    const T* src = gathered + L.gathered_index(i, rows_per_rank) * row_len;
    std::copy(src, src + row_len, out + static_cast<size_t>(i) * row_len);
  }
}

// Per-item success from the ranks' gathered shard flags (flag != 0: that rank's forward ran): an
// item fails exactly when the rank that computed it failed.
inline std::vector<uint8_t> dp_item_ok(const DpLayout& L, const int* rank_ok) {
  std::vector<uint8_t> ok(static_cast<size_t>(L.B), 1);
  for (int i = 0; i < L.B; ++i) ok[static_cast<size_t>(i)] = rank_ok[L.rank_of(i)] != 0;
  return ok;
}

}  // namespace die
