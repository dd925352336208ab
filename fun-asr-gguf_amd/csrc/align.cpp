// Host-side char-timestamp alignment (A14), bit-identical to the reference's Python
// align_timestamps (/root/reference/fun_asr_gguf/nano_ctc.py:118-232):
//   global Needleman-Wunsch, match +1 / mismatch -1 / gap -1, case-insensitive (the caller maps each
//   char's .lower() string to an integer key), tie order diag > up > left (:167-172), traceback
//   (:176-191), then linear interpolation of unaligned chars between anchors, +0.05 s after the last
//   anchor, max(0, next - 0.05) before the first (:193-226).
// Scores are small integers (exact in the reference's float32 matrix), kept as int32 here. Double
// arithmetic follows the Python evaluation order; this file is compiled with -ffp-contract=off.
#include <stdint.h>

#include <vector>

#include "../../include/funasr_hip.h"

extern "C" int fa_align_timestamps(const int32_t* ctc_keys, const double* ctc_starts, int32_t n_ctc,
                                   const int32_t* llm_keys, int32_t n_llm, double* starts_out, int32_t* aligned_out) {
  if (n_ctc <= 0 || n_llm <= 0) return FA_OK;  // reference returns [] (caller handles)
  if (!ctc_keys || !ctc_starts || !llm_keys || !starts_out) return FA_ERR_ARG;
  const int n = n_ctc + 1, m = n_llm + 1;
  std::vector<int32_t> prev(m), cur(m);
  std::vector<uint8_t> trace((size_t)n * m, 0);
  for (int j = 0; j < m; ++j) prev[j] = -j;
  for (int i = 1; i < n; ++i) {
    cur[0] = -i;
    const int32_t a = ctc_keys[i - 1];
    uint8_t* tr = &trace[(size_t)i * m];
    for (int j = 1; j < m; ++j) {
      const int32_t d = prev[j - 1] + (a == llm_keys[j - 1] ? 1 : -1);
      const int32_t u = prev[j] - 1;
      const int32_t l = cur[j - 1] - 1;
      int32_t best = d > u ? d : u;
      best = best > l ? best : l;
      cur[j] = best;
      tr[j] = best == d ? 1 : (best == u ? 2 : 3);
    }
    prev.swap(cur);
  }
  std::vector<int32_t> al(n_llm, -1);  // index of the aligned ctc char or -1
  int i = n - 1, j = m - 1;
  while (i > 0 || j > 0) {
    const uint8_t t = trace[(size_t)i * m + j];
    if (i > 0 && j > 0 && t == 1) {
      al[j - 1] = i - 1;
      --i;
      --j;
    } else if (i > 0 && (j == 0 || t == 2)) {
      --i;
    } else if (j > 0 && (i == 0 || t == 3)) {
      al[j - 1] = -1;
      --j;
    } else {
      break;  // unreachable for a well-formed trace
    }
  }
  // anchors in index order; prev/next anchor for every position
  std::vector<int> prev_a(n_llm, -1), next_a(n_llm, -1);
  int last = -1;
  for (int k = 0; k < n_llm; ++k) {
    prev_a[k] = last;  // strictly before k
    if (al[k] >= 0) last = k;
  }
  last = -1;
  for (int k = n_llm - 1; k >= 0; --k) {
    next_a[k] = last;  // strictly after k
    if (al[k] >= 0) last = k;
  }
  for (int k = 0; k < n_llm; ++k) {
    if (aligned_out) aligned_out[k] = al[k];
    if (al[k] >= 0) {
      starts_out[k] = ctc_starts[al[k]];
      continue;
    }
    const int pa = prev_a[k], na = next_a[k];
    if (pa >= 0 && na >= 0) {
      const double p_start = ctc_starts[al[pa]], n_start = ctc_starts[al[na]];
      const double step = (n_start - p_start) / (double)(na - pa);
      starts_out[k] = p_start + (double)(k - pa) * step;
    } else if (pa >= 0) {
      starts_out[k] = ctc_starts[al[pa]] + 0.05;
    } else if (na >= 0) {
      const double v = ctc_starts[al[na]] - 0.05;
      starts_out[k] = v < 0.0 ? 0.0 : v;
    } else {
      starts_out[k] = 0.0;
    }
  }
  return FA_OK;
}

// FastRAG coarse retrieval distance (/root/reference/fun_asr_gguf/hotword/rag_fast.py:35-77, the numba kernel):
// minimum over end positions j >= 1 of the edit distance between the hotword's phoneme codes (sub) and a
// substring of the input's codes (main) ending at j, free start (dp[0][j] = 0), unit insert / delete / substitute.
// Float32 DP as in the reference (all values are small integers: exact).
extern "C" int fa_fuzzy_substring_distance(const int32_t* main_codes, int32_t m, const int32_t* sub_codes, int32_t n,
                                           float* dist_out) {
  if (!dist_out || m < 0 || n < 0) return FA_ERR_ARG;
  if (n == 0 || m == 0) {
    *dist_out = (float)n;
    return FA_OK;
  }
  if (!main_codes || !sub_codes) return FA_ERR_ARG;
  std::vector<float> prev(m + 1, 0.f), cur(m + 1);
  for (int i = 1; i <= n; ++i) {
    cur[0] = (float)i;
    const int32_t s = sub_codes[i - 1];
    for (int j = 1; j <= m; ++j) {
      const float cost = s == main_codes[j - 1] ? 0.f : 1.f;
      float v = prev[j] + 1.f;
      if (cur[j - 1] + 1.f < v) v = cur[j - 1] + 1.f;
      if (prev[j - 1] + cost < v) v = prev[j - 1] + cost;
      cur[j] = v;
    }
    prev.swap(cur);
  }
  float best = prev[1];
  for (int j = 2; j <= m; ++j)
    if (prev[j] < best) best = prev[j];
  *dist_out = best;
  return FA_OK;
}
