// CPU rule-index matcher: exact reference semantics of recommend_tracks_for_track
// (rest_api/app/main.py:224-254) over an integer CSR index instead of dict-of-dicts.
//
//   present  = seeds that are keys, request order (duplicates kept)
//   merged   = insertion-ordered map, merged[r] = max(merged[r], score)
//   output   = stable sort by score desc (ties: insertion order), first k
//
// Per-thread scratch uses epoch stamps so a query costs O(Σ row length + k log k), not O(I).
#include <algorithm>
#include <vector>

#include "kmls/host.hpp"

namespace kmls {

RuleIndex::RuleIndex(int64_t n_items, std::vector<int64_t> row_ptr, std::vector<int32_t> cons,
                     std::vector<double> score, std::vector<uint8_t> is_key)
    : n_items_(n_items), row_ptr_(std::move(row_ptr)), cons_(std::move(cons)),
      score_(std::move(score)), is_key_(std::move(is_key)) {
  KMLS_CHECK((int64_t)row_ptr_.size() == n_items_ + 1, "row_ptr size mismatch");
  KMLS_CHECK((int64_t)is_key_.size() == n_items_, "is_key size mismatch");
  KMLS_CHECK(cons_.size() == score_.size(), "cons/score size mismatch");
  KMLS_CHECK(row_ptr_.back() == (int64_t)cons_.size(), "row_ptr/nnz mismatch");
  for (int32_t c : cons_) KMLS_CHECK(c >= 0 && c < n_items_, "consequent out of range");
}

namespace {
struct Scratch {
  std::vector<uint32_t> stamp;  // epoch of last touch
  std::vector<double> val;
  std::vector<uint32_t> seq;
  std::vector<int32_t> touched;
  uint32_t epoch = 0;
  void ensure(int64_t n) {
    if ((int64_t)stamp.size() < n) {
      stamp.assign((size_t)n, 0);
      val.resize((size_t)n);
      seq.resize((size_t)n);
      epoch = 0;
    }
    if (++epoch == 0) {  // wrapped: reset
      std::fill(stamp.begin(), stamp.end(), 0);
      epoch = 1;
    }
    touched.clear();
  }
};
thread_local Scratch tls;
}  // namespace

int RuleIndex::query(const int32_t* seeds, int n_seeds, int k, int32_t* out_ids,
                     double* out_scores) const {
  bool any = false;
  for (int s = 0; s < n_seeds; ++s) {
    int32_t q = seeds[s];
    if (q >= 0 && q < n_items_ && is_key_[q]) { any = true; break; }
  }
  if (!any) return -1;
  Scratch& sc = tls;
  sc.ensure(n_items_);
  const uint32_t ep = sc.epoch;
  uint32_t next_seq = 0;
  for (int s = 0; s < n_seeds; ++s) {
    int32_t q = seeds[s];
    if (q < 0 || q >= n_items_ || !is_key_[q]) continue;
    for (int64_t p = row_ptr_[q]; p < row_ptr_[q + 1]; ++p) {
      const int32_t r = cons_[p];
      const double v = score_[p];
      if (sc.stamp[r] != ep) {
        sc.stamp[r] = ep;
        sc.val[r] = v > 0.0 ? v : 0.0;  // defaultdict(int) starts at 0
        sc.seq[r] = next_seq++;
        sc.touched.push_back(r);
      } else if (v > sc.val[r]) {
        sc.val[r] = v;
      }
    }
  }
  const int n = (int)sc.touched.size();
  const int kk = std::min(k, n);
  auto better = [&](int32_t a, int32_t b) {
    if (sc.val[a] != sc.val[b]) return sc.val[a] > sc.val[b];
    return sc.seq[a] < sc.seq[b];
  };
  std::partial_sort(sc.touched.begin(), sc.touched.begin() + kk, sc.touched.end(), better);
  for (int i = 0; i < kk; ++i) {
    out_ids[i] = sc.touched[i];
    if (out_scores) out_scores[i] = sc.val[sc.touched[i]];
  }
  return kk;
}

}  // namespace kmls
