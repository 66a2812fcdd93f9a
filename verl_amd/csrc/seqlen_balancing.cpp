// Host-side sequence-length balancing for the actor path: the largest-differencing-method
// (Karmarkar-Karp) k-way partition the reference uses to (a) reorder a batch so every DP rank
// gets a similar token count (ray_trainer.py:1064-1079 `_balance_batch`) and (b) cut dynamic
// token-budget micro-batches (seqlen_balancing.py:239-300 `rearrange_micro_batches`).
//
// Reference algorithm: verl/utils/seqlen_balancing.py:26-127. It runs once per batch / per
// mini-batch on the host (Python, O(n k log k) object comparisons); this is the same algorithm in
// C++ so it stays off the step's critical path at n = 512, k = 64.
//
// Result parity with the reference is exact, not approximate:
//   * a partition ("set") orders by (sum, item count, item list lexicographic by (index, value));
//     two distinct states never compare equal (their largest sets hold different indices), so any
//     correct priority queue pops states in the reference's order;
//   * inside a state the sets are kept in descending order by a STABLE sort, as Python's
//     `sorted(..., reverse=True)`;
//   * merging pairs set i of the popped state with set k-1-i of the second state, appending
//     items in their existing order.

#include <stdint.h>

#include <algorithm>
#include <queue>
#include <utility>
#include <vector>

#include "../../include/verl_amd.h"

namespace {

struct Part {
  int64_t sum = 0;
  std::vector<std::pair<int64_t, int64_t>> items;  // (index, value) in insertion order
};

// strict "a orders before b" for partitions
bool part_less(const Part &a, const Part &b) {
  if (a.sum != b.sum) return a.sum < b.sum;
  if (a.items.size() != b.items.size()) return a.items.size() < b.items.size();
  return a.items < b.items;
}

struct State {
  std::vector<Part> parts;  // descending
  int64_t spread() const { return parts.front().sum - parts.back().sum; }
  void sort_desc() {
    std::stable_sort(parts.begin(), parts.end(), [](const Part &a, const Part &b) { return part_less(b, a); });
  }
};

// heap order: the state with the largest spread first; on equal spread the one whose largest
// partition is larger
struct PopsLater {
  const std::vector<State> *pool;
  bool operator()(int a, int b) const {  // true when a pops after b
    const State &x = (*pool)[a], &y = (*pool)[b];
    const int64_t sx = x.spread(), sy = y.spread();
    if (sx != sy) return sx < sy;
    return part_less(x.parts.front(), y.parts.front());
  }
};

}  // namespace

extern "C" int va_karmarkar_karp(const int64_t *seqlens, int64_t n, int64_t k, int equal_size, int64_t *order,
                                 int64_t *offsets) {
  if (n < 0 || k <= 0 || (n > 0 && (seqlens == nullptr || order == nullptr)) || offsets == nullptr) return VA_E_ARG;
  if (equal_size && n % k != 0) return VA_E_ARG;
  if (n == 0) {
    for (int64_t i = 0; i <= k; ++i) offsets[i] = 0;
    return VA_OK;
  }
  // items sorted ascending by (value, index)
  std::vector<std::pair<int64_t, int64_t>> sorted(n);
  for (int64_t i = 0; i < n; ++i) sorted[i] = {seqlens[i], i};
  std::sort(sorted.begin(), sorted.end());

  std::vector<State> pool;
  pool.reserve(equal_size ? n / k : n);
  auto new_state = [&](int64_t first, int64_t count) {
    State s;
    s.parts.resize(k);
    for (int64_t j = 0; j < count; ++j) {
      s.parts[j].items.push_back({sorted[first + j].second, sorted[first + j].first});
      s.parts[j].sum = sorted[first + j].first;
    }
    s.sort_desc();
    pool.push_back(std::move(s));
  };
  if (equal_size) {
    for (int64_t off = 0; off < n; off += k) new_state(off, k);
  } else {
    for (int64_t i = 0; i < n; ++i) new_state(i, 1);
  }
  PopsLater cmp{&pool};
  std::priority_queue<int, std::vector<int>, PopsLater> pq(cmp);
  for (int i = 0; i < static_cast<int>(pool.size()); ++i) pq.push(i);
  while (pq.size() > 1) {
    const int a = pq.top();
    pq.pop();
    const int b = pq.top();
    pq.pop();
    State &x = pool[a];
    State &y = pool[b];
    for (int64_t i = 0; i < k; ++i) {
      Part &dst = x.parts[i];
      Part &src = y.parts[k - 1 - i];
      dst.items.insert(dst.items.end(), src.items.begin(), src.items.end());
      dst.sum += src.sum;
    }
    y.parts.clear();
    y.parts.shrink_to_fit();
    x.sort_desc();
    pq.push(a);
  }
  const State &fin = pool[pq.top()];
  int64_t pos = 0;
  for (int64_t i = 0; i < k; ++i) {
    offsets[i] = pos;
    for (const auto &it : fin.parts[i].items) order[pos++] = it.first;
  }
  offsets[k] = pos;
  return VA_OK;
}
