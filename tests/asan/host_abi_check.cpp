// Host-side checks of the C-ABI under AddressSanitizer + UndefinedBehaviorSanitizer
// ("CPU sanitizer build").  TEST INFRASTRUCTURE ONLY.
//
// The library's host code -- argument validation of every entry point, the attention work
// planner cs_prefix_attention_plan (std::vector cells written through a caller's int32
// buffer), the split / workspace planners -- and the C oracle are compiled host-only with
// -fsanitize=address,undefined (tests/asan/Makefile) and driven here without a GPU: only
// calls that must return before any launch (bad arguments, empty shapes, pure host
// functions).  Any out-of-bounds access, overflow or UB aborts the binary; the checks
// below abort on a wrong answer.  Run by tests/test_sanitizers.py.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "consensus_scoring.h"

extern "C" {
// oracle/cs_oracle.c
void oracle_logsoftmax_gather(const void* logits, int dtype, int64_t rows, int64_t vocab,
                              int64_t ld, const int32_t* target_ids, int32_t k, double softcap,
                              double* out_tok_lp, double* out_lse);
void oracle_segment_reduce(const double* tok_lp, const int32_t* seg_offsets, int64_t n_seg,
                           double* out_sum_lp, double* out_sum_p, int32_t* out_count,
                           double* out_last);
void oracle_welfare(const double* U, int32_t A, int32_t C, int64_t ldu, int kind, double eps,
                    int nonfinite, double nan_val, double posinf_val, double neginf_val,
                    double* W);
void oracle_topk(const double* W, int32_t n_seg, int32_t seg_len, int64_t ld, int32_t k,
                 int32_t* out_idx);
}

static int g_fail = 0;
#define CHECK(cond, ...)                                        \
  do {                                                          \
    if (!(cond)) {                                              \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                        \
      std::fprintf(stderr, "\n");                               \
      ++g_fail;                                                 \
    }                                                           \
  } while (0)

// an argument error: negative status and a message
#define REJECTS(call) CHECK((call) < 0 && std::strlen(cs_last_error()) > 0, "not rejected: %s", #call)

// ---------------------------------------------------------------------------------------
// cs_prefix_attention_plan: every entry within the documented ranges, slots and merge
// chunks consistent with the workspace size, exact-size buffers (ASan bounds)
static void check_plan(std::mt19937_64& rng, int iters) {
  int planned = 0;
  for (int it = 0; it < iters; ++it) {
    const int D = std::vector<int>{64, 128, 256}[rng() % 3];
    const int Hkv = 1 + static_cast<int>(rng() % 8);
    const int rep = 1 + static_cast<int>(rng() % 8);
    const int H = Hkv * rep;
    const int n_prefix = 1 + static_cast<int>(rng() % 70);
    const int n_groups = 1 + static_cast<int>(rng() % 70);
    const int n_str = 1 + static_cast<int>(rng() % 64);
    const int T = (rng() % 4) ? 1 : 1 + static_cast<int>(rng() % 160);
    const int64_t ld_hist = 32 * (1 + static_cast<int64_t>(rng() % 8));
    std::vector<int32_t> plen(n_prefix), gpfx(n_groups);
    for (auto& p : plen) p = static_cast<int32_t>(rng() % ((rng() % 8) ? 400 : 6000));
    for (auto& g : gpfx) g = static_cast<int32_t>(rng() % n_prefix);
    const bool ident = n_groups <= n_prefix && (rng() % 2);
    int32_t na = -1, nm = -1;
    size_t ws = 1;
    const int64_t total = cs_prefix_attention_plan(plen.data(), n_prefix, ident ? nullptr : gpfx.data(),
                                                   n_groups, n_str, T, H, Hkv, D, ld_hist, nullptr, 0,
                                                   &na, &nm, &ws);
    CHECK(total >= 0, "plan sizing failed: %s", cs_last_error());
    if (total <= 0) {
      CHECK(na == 0 && nm == 0 && ws == 0, "no plan but counts set");
      continue;
    }
    ++planned;
    CHECK(total == static_cast<int64_t>(na) + nm, "total %lld != %d + %d", (long long)total, na, nm);
    std::vector<int32_t> plan(static_cast<size_t>(4 * total));   // exact: ASan catches overruns
    CHECK(cs_prefix_attention_plan(plen.data(), n_prefix, ident ? nullptr : gpfx.data(), n_groups,
                                   n_str, T, H, Hkv, D, ld_hist, plan.data(), total - 1, nullptr,
                                   nullptr, nullptr) < 0,
          "plan_cap too small accepted");
    const int64_t again = cs_prefix_attention_plan(plen.data(), n_prefix, ident ? nullptr : gpfx.data(),
                                                   n_groups, n_str, T, H, Hkv, D, ld_hist, plan.data(),
                                                   total, nullptr, nullptr, nullptr);
    CHECK(again == total, "fill returned %lld", (long long)again);
    const int64_t M = static_cast<int64_t>(n_str) * T * rep;
    const int64_t n_qg = (M + 63) / 64;
    const int64_t slot_bytes = 64 * (D + 2) * static_cast<int64_t>(sizeof(float));
    CHECK(ws % slot_bytes == 0, "workspace %zu not a whole number of slots", ws);
    const int64_t n_slots = static_cast<int64_t>(ws) / slot_bytes;
    std::vector<int> slot_used(static_cast<size_t>(n_slots), 0);
    for (int64_t e = 0; e < na; ++e) {
      const int32_t* p = &plan[4 * e];
      const int split = p[2] & 255, n_used = p[2] >> 8;
      CHECK(p[0] >= 0 && p[0] < n_groups * Hkv, "attn pg %d", p[0]);
      CHECK(p[1] >= 0 && p[1] < n_qg, "attn qg %d", p[1]);
      CHECK(n_used >= 1 && n_used <= 32 && split < n_used, "attn split %d / %d", split, n_used);
      if (n_used > 1) {
        CHECK(p[3] >= 0 && p[3] < n_slots, "attn slot %d of %lld", p[3], (long long)n_slots);
        if (p[3] >= 0 && p[3] < n_slots) slot_used[p[3]]++;
      }
    }
    for (int64_t s = 0; s < n_slots; ++s) CHECK(slot_used[s] == 1, "slot %lld written %d times", (long long)s, slot_used[s]);
    for (int64_t e = na; e < total; ++e) {
      const int32_t* p = &plan[4 * e];
      const int n_used = p[3] >> 8, ch = p[3] & 255;
      CHECK(p[0] >= 0 && p[0] < n_groups * Hkv && p[1] >= 0 && p[1] < n_qg, "merge cell");
      CHECK(n_used > 1 && p[2] >= 0 && p[2] + n_used <= n_slots, "merge slots %d + %d", p[2], n_used);
      CHECK(ch >= 0 && ch < 8, "merge chunk %d", ch);
    }
  }
  CHECK(planned > iters / 20, "only %d of %d shapes planned", planned, iters);
  // bad shapes
  const int32_t pl[2] = {10, 20};
  const int32_t bad_g[1] = {5};
  REJECTS(cs_prefix_attention_plan(pl, 2, bad_g, 1, 4, 1, 8, 2, 64, 32, nullptr, 0, nullptr, nullptr, nullptr));
  REJECTS(cs_prefix_attention_plan(pl, 2, nullptr, 1, 4, 1, 8, 3, 64, 32, nullptr, 0, nullptr, nullptr, nullptr));
  REJECTS(cs_prefix_attention_plan(pl, 2, nullptr, 1, 4, 1, 8, 2, 96, 32, nullptr, 0, nullptr, nullptr, nullptr));
  REJECTS(cs_prefix_attention_plan(pl, 2, nullptr, 1, 4, 1, 8, 2, 64, 40, nullptr, 0, nullptr, nullptr, nullptr));
  REJECTS(cs_prefix_attention_plan(nullptr, 2, nullptr, 1, 4, 1, 8, 2, 64, 32, nullptr, 0, nullptr, nullptr, nullptr));
  REJECTS(cs_prefix_attention_plan(pl, 2, nullptr, -1, 4, 1, 8, 2, 64, 32, nullptr, 0, nullptr, nullptr, nullptr));
  CHECK(cs_prefix_attention_plan(pl, 2, nullptr, 0, 4, 1, 8, 2, 64, 32, nullptr, 0, nullptr, nullptr, nullptr) == 0,
        "empty plan");
}

// ---------------------------------------------------------------------------------------
// pure-host planners at ordinary and extreme sizes (UBSan: no signed overflow)
static void check_planners(std::mt19937_64& rng, int iters) {
  const int64_t big[] = {0, 1, 7, 4096, 128256, 256000, int64_t{1} << 31, int64_t{1} << 40};
  for (int64_t rows : big)
    for (int64_t V : big) {
      (void)cs_workspace_size(rows, V, 1);
      (void)cs_workspace_size(rows, V, 64);
      (void)cs_beam_step_workspace_size(rows, V);
      (void)cs_vocab_topk_workspace_size(rows, V, 16);
      (void)cs_vocab_sample_workspace_size(rows, V, 4);
    }
  for (int it = 0; it < iters; ++it) {
    const int32_t A = 1 + static_cast<int32_t>(rng() % 64), B = 1 + static_cast<int32_t>(rng() % 16);
    const int64_t V = 1 + static_cast<int64_t>(rng() % 300000);
    const int32_t K = 1 + static_cast<int32_t>(rng() % 64);
    (void)cs_beam_decode_workspace_size(A, B, V, K);
    const int64_t M = 1 + static_cast<int64_t>(rng() % 4096);
    const int64_t N = 128 * (1 + static_cast<int64_t>(rng() % 1024));
    const int64_t Kd = 64 * (1 + static_cast<int64_t>(rng() % 512));
    for (int variant = 0; variant <= 7; ++variant)
      for (int gated = 0; gated <= 1; ++gated) {
        const int64_t s = cs_gemm_splits(M, N, Kd, gated, variant);
        CHECK(s >= 0 && s <= Kd / 64, "cs_gemm_splits %lld", (long long)s);
        if (gated || variant >= 5) CHECK(s <= 1, "a gated / thin GEMM split %lld", (long long)s);
      }
  }
  CHECK(cs_gemm_splits(8, 100, 64, 0, 2) == 0, "N %% 128 accepted");
}

// ---------------------------------------------------------------------------------------
// every compute entry rejects bad arguments before it launches, and returns 0 on empty work
static void check_rejections() {
  void* d = reinterpret_cast<void*>(uintptr_t{256});
  float* f = reinterpret_cast<float*>(uintptr_t{256});
  int32_t* i = reinterpret_cast<int32_t*>(uintptr_t{256});
  REJECTS(cs_logsoftmax_gather(nullptr, 0, 4, 128, 128, i, 1, 0.f, f, nullptr, nullptr, 0, nullptr));
  REJECTS(cs_logsoftmax_gather(d, 0, -1, 128, 128, i, 1, 0.f, f, nullptr, nullptr, 0, nullptr));
  REJECTS(cs_logsoftmax_gather(d, 0, 4, 128, 64, i, 1, 0.f, f, nullptr, nullptr, 0, nullptr));
  REJECTS(cs_logsoftmax_gather(d, 7, 4, 128, 128, i, 1, 0.f, f, nullptr, nullptr, 0, nullptr));
  CHECK(cs_logsoftmax_gather(d, 0, 0, 128, 128, i, 1, 0.f, f, nullptr, nullptr, 0, nullptr) == 0, "empty lsg");
  REJECTS(cs_segment_reduce(f, -1, i, 1, f, nullptr, nullptr, nullptr, nullptr));
  REJECTS(cs_segment_reduce(f, 4, nullptr, 1, f, nullptr, nullptr, nullptr, nullptr));
  REJECTS(cs_welfare_reduce(nullptr, 2, 4, 4, 0, 0.f, 0, 0.f, 0.f, 0.f, f, nullptr));
  REJECTS(cs_welfare_reduce(f, 2, 4, 2, 0, 0.f, 0, 0.f, 0.f, 0.f, f, nullptr));
  REJECTS(cs_welfare_reduce(f, 2, 4, 4, 9, 0.f, 0, 0.f, 0.f, 0.f, f, nullptr));
  REJECTS(cs_segmented_topk(f, 1, 8, 8, 9, i, nullptr, nullptr));
  REJECTS(cs_segmented_topk(f, 1, 8, 4, 2, i, nullptr, nullptr));
  REJECTS(cs_segmented_topk(nullptr, 1, 8, 8, 2, i, nullptr, nullptr));
  REJECTS(cs_vocab_topk(d, 0, 2, 128, 128, 300, 0.f, i, nullptr, d, 1 << 20, nullptr));
  REJECTS(cs_vocab_topk(nullptr, 0, 2, 128, 128, 4, 0.f, i, nullptr, d, 1 << 20, nullptr));
  REJECTS(cs_vocab_sample(d, 0, 2, 128, 128, 1.f, 0.f, nullptr, 1, i, nullptr, d, 1 << 20, nullptr));
  REJECTS(cs_vocab_sample(d, 0, 2, 128, 128, 1.f, 0.f, reinterpret_cast<const uint64_t*>(d), 17, i,
                          nullptr, d, 1 << 20, nullptr));
  REJECTS(cs_beam_step(d, 0, 2, 2, 128, 128, nullptr, 4, f, 0.f, 0, 0.f, f, f, 0, nullptr, nullptr,
                       nullptr, d, 1 << 20, nullptr));
  REJECTS(cs_beam_step(d, 0, 2, 2, 128, 128, i, 4, f, 0.f, 0, 0.f, f, f, 0, nullptr, nullptr,
                       nullptr, nullptr, 0, nullptr));
  REJECTS(cs_beam_decode_step(d, 128, d, 128, 0, 2, 2, 128, 300, 0.f, f, 0, 0.f, i, f, f, 0,
                              nullptr, nullptr, nullptr, d, 1 << 20, nullptr));
  REJECTS(cs_beam_select(f, 2048, 0, f, 2, 4, nullptr, i, nullptr, nullptr, nullptr));
  REJECTS(cs_beam_select(f, 16, 0, f, 2, 0, nullptr, i, nullptr, nullptr, nullptr));
  const int64_t off[1] = {0};
  const int32_t pl[1] = {8};
  REJECTS(cs_prefix_attention(d, d, d, 32, off, pl, 8, nullptr, 1, d, d, 32, i, 4, 1, 8, 3, 64, 0.1f,
                              0.f, 0, nullptr, 0, 0, d, nullptr, 0, nullptr));
  REJECTS(cs_prefix_attention(d, d, d, 32, off, pl, 8, nullptr, 1, d, d, 32, i, 4, 1, 8, 2, 80, 0.1f,
                              0.f, 0, nullptr, 0, 0, d, nullptr, 0, nullptr));
  REJECTS(cs_prefix_attention(d, d, d, 32, off, pl, 40, nullptr, 1, d, d, 32, i, 4, 1, 8, 2, 64, 0.1f,
                              0.f, 0, nullptr, 0, 0, d, nullptr, 0, nullptr));
  REJECTS(cs_prefix_attention(d, d, d, 32, off, pl, 8, nullptr, 1, d, d, 32, i, 4, 1, 8, 2, 64, 0.1f,
                              0.f, 0, d, 4, 1, d, nullptr, 0, nullptr));
  CHECK(cs_prefix_attention(d, d, d, 32, off, pl, 8, nullptr, 0, d, d, 32, i, 4, 1, 8, 2, 64, 0.1f, 0.f,
                            0, nullptr, 0, 0, d, nullptr, 0, nullptr) == 0,
        "empty attention");
  REJECTS(cs_gemm_bf16(d, 64, d, 64, d, 128, 4, 100, 64, 1, 0, 0, 2, nullptr, nullptr));
  REJECTS(cs_gemm_bf16(d, 64, d, 64, d, 128, 4, 128, 96, 1, 0, 0, 2, nullptr, nullptr));
  REJECTS(cs_gemm_bf16(nullptr, 64, d, 64, d, 128, 4, 128, 64, 1, 0, 0, 2, nullptr, nullptr));
  REJECTS(cs_gemm_bf16(d, 64, d, 64, d, 128, 81, 128, 64, 1, 0, 0, 5, nullptr, nullptr));
  REJECTS(cs_gemm_bf16_packed(d, 64, d, d, 128, 4, 128, 64, 1, 0, 0, 5, nullptr, nullptr));
  REJECTS(cs_gemm_pack(d, 64, 24, 64, d, nullptr));
  REJECTS(cs_gemm_pack(reinterpret_cast<void*>(uintptr_t{260}), 64, 32, 64, d, nullptr));
  REJECTS(cs_add_rms_norm(nullptr, 64, nullptr, 0, nullptr, d, 64, d, 4, 64, 1e-6f, 0, d, 64, nullptr));
  REJECTS(cs_add_rms_norm(d, 64, nullptr, 0, nullptr, d, 64, d, 4, 60, 1e-6f, 0, d, 64, nullptr));
  REJECTS(cs_add_rms_norm_splitk(d, 64, f, 17, nullptr, d, 64, d, 4, 64, 1e-6f, 0, d, 64, nullptr));
  REJECTS(cs_gated_act(d, 64, d, 64, -1, 64, 0, d, 64, nullptr));
  REJECTS(cs_gated_act(d, 64, d, 64, 4, 60, 0, d, 64, nullptr));
  const int64_t* par = reinterpret_cast<const int64_t*>(d);
  REJECTS(cs_rope_place(nullptr, 64, f, i, nullptr, 1, i, 1, 1, 1, 1, 64, d, d, d, 32, nullptr));
  REJECTS(cs_rope_place_splitk(f, 2, f, i, nullptr, 1, i, 1, 32, 4, 2, 64, d, d, d, 64, nullptr));
  // the row-layout history entries
  REJECTS(cs_prefix_attention_rows(d, d, d, 32, off, pl, 8, nullptr, 1, d, d, nullptr, 32, i, 4, 1, 8,
                                   2, 64, 0.1f, 0.f, 0, nullptr, 0, 0, d, nullptr, 0, nullptr));
  REJECTS(cs_prefix_attention_rows(d, d, d, 32, off, pl, 8, nullptr, 1, d, d, i, 40, i, 4, 1, 8, 2, 64,
                                   0.1f, 0.f, 0, nullptr, 0, 0, d, nullptr, 0, nullptr));
  REJECTS(cs_rope_place_rows(nullptr, 64, f, i, nullptr, 1, i, 1, 1, 1, 1, 64, d, d, d, 32, nullptr));
  REJECTS(cs_rope_place_splitk_rows(f, 2, f, i, nullptr, 1, i, 1, 32, 4, 2, 64, d, d, d, 64, nullptr));
  REJECTS(cs_hist_rows_update(i, i, par, i, 4, 32, 0, 4, nullptr));       // source == destination
  REJECTS(cs_hist_rows_update(i, i + 1, par, i, 4, 32, -1, 4, nullptr));  // negative row base
  REJECTS(cs_hist_rows_update(nullptr, i, par, i, 4, 32, 0, 4, nullptr));
  REJECTS(cs_hist_rows_update(i, i + 1, par, i, 4, 32, 0, 3, nullptr));   // rows past the buffer
  REJECTS(cs_hist_rows_update(i, i + 1, par, i, 4, 32, 2, 5, nullptr));   // row_base + S > n_rows
  CHECK(cs_hist_rows_update(i, i + 1, par, i, 0, 32, 0, 0, nullptr) == 0, "empty rows update");
}

// ---------------------------------------------------------------------------------------
// the C oracle under the sanitizers: known answers from a direct fp64 restatement
static uint16_t to_bf16(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  return static_cast<uint16_t>((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

static void check_oracle(std::mt19937_64& rng) {
  std::normal_distribution<float> nd(0.f, 3.f);
  const int64_t rows = 5, V = 1000, ld = 1003;
  const int32_t k = 3;
  std::vector<float> lf(static_cast<size_t>(rows * ld));
  std::vector<uint16_t> lb(lf.size());
  for (size_t j = 0; j < lf.size(); ++j) {
    lb[j] = to_bf16(nd(rng));
    const uint32_t u = static_cast<uint32_t>(lb[j]) << 16;
    std::memcpy(&lf[j], &u, 4);   // the bf16 values exactly, as fp32
  }
  std::vector<int32_t> tg(static_cast<size_t>(rows * k));
  for (auto& t : tg) t = static_cast<int32_t>(rng() % (V + 2)) - 1;   // incl. -1 and V (NaN)
  for (double cap : {0.0, 30.0}) {
    std::vector<double> lp32(rows * k), lp16(rows * k), lse(rows);
    oracle_logsoftmax_gather(lf.data(), 0, rows, V, ld, tg.data(), k, cap, lp32.data(), lse.data());
    oracle_logsoftmax_gather(lb.data(), 1, rows, V, ld, tg.data(), k, cap, lp16.data(), nullptr);
    for (int64_t r = 0; r < rows; ++r) {
      double s = 0.0;
      for (int64_t v = 0; v < V; ++v) {
        const double x = lf[r * ld + v];
        s += std::exp(cap > 0 ? cap * std::tanh(x / cap) : x);
      }
      CHECK(std::fabs(std::log(s) - lse[r]) < 1e-9, "lse row %lld", (long long)r);
      for (int j = 0; j < k; ++j) {
        const int32_t t = tg[r * k + j];
        const double a = lp32[r * k + j], b = lp16[r * k + j];
        if (t < 0 || t >= V) {
          CHECK(std::isnan(a) && std::isnan(b), "out-of-range target not NaN");
        } else {
          const double x = lf[r * ld + t];
          const double want = (cap > 0 ? cap * std::tanh(x / cap) : x) - std::log(s);
          CHECK(std::fabs(a - want) < 1e-9 && a == b, "lp row %lld target %d", (long long)r, t);
        }
      }
    }
  }
  // segments (incl. empty) and NaN skipping
  const double tl[7] = {-1.0, NAN, -2.0, -0.5, NAN, -3.0, -0.25};
  const int32_t so[5] = {0, 3, 3, 5, 7};
  double sl[4], sp[4], last[4];
  int32_t cnt[4];
  oracle_segment_reduce(tl, so, 4, sl, sp, cnt, last);
  CHECK(sl[0] == -3.0 && cnt[0] == 2 && last[0] == -2.0, "segment 0");
  CHECK(sl[1] == 0.0 && cnt[1] == 0 && std::isnan(last[1]), "empty segment");
  CHECK(sl[2] == -0.5 && cnt[2] == 1 && std::isnan(last[2]), "segment 2");
  CHECK(sl[3] == -3.25 && cnt[3] == 2 && last[3] == -0.25, "segment 3");
  CHECK(std::fabs(sp[3] - (std::exp(-3.0) + std::exp(-0.25))) < 1e-15, "segment 3 sum p");
  // welfare kinds over agents, skip / replace
  const double U[6] = {-1.0, NAN, 0.5, -2.0, 3.0, INFINITY};   // [A = 2][C = 3]
  double W[3];
  oracle_welfare(U, 2, 3, 3, 0, 1e-9, 0, 0, 0, 0, W);
  CHECK(W[0] == -2.0 && W[1] == 3.0 && W[2] == 0.5, "min skip");
  oracle_welfare(U, 2, 3, 3, 0, 1e-9, 1, -10.0, 20.0, -20.0, W);
  CHECK(W[0] == -2.0 && W[1] == -10.0 && W[2] == 0.5, "min replace");
  oracle_welfare(U, 2, 3, 3, 1, 1e-9, 0, 0, 0, 0, W);
  CHECK(W[0] == -3.0 && W[1] == 3.0 && W[2] == 0.5, "sum skip");
  oracle_welfare(U, 2, 3, 3, 2, 1e-9, 0, 0, 0, 0, W);
  CHECK(std::fabs(W[0] - 2 * std::log(1e-9)) < 1e-9 && std::fabs(W[2] - std::log(0.5)) < 1e-15, "sumlog");
  // top-k: stable descending order, NaN last, against std::stable_sort
  for (int it = 0; it < 20; ++it) {
    const int32_t L = 1 + static_cast<int32_t>(rng() % 300), kk = 1 + static_cast<int32_t>(rng() % L);
    std::vector<double> w(L);
    for (auto& x : w) x = (rng() % 10 == 0) ? NAN : static_cast<double>(rng() % 7);   // ties
    std::vector<int32_t> got(kk), ord(L);
    oracle_topk(w.data(), 1, L, L, kk, got.data());
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) {
      if (std::isnan(w[a]) || std::isnan(w[b])) return !std::isnan(w[a]) && std::isnan(w[b]);
      return w[a] > w[b];
    });
    CHECK(std::equal(got.begin(), got.end(), ord.begin()), "top-k order (L %d, k %d)", L, kk);
  }
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "overflow") == 0) {   // the build IS sanitized
    std::vector<int32_t> v(4);
    int32_t* p = v.data();
    volatile int at = 4;
    p[at] = 1;
    return 0;
  }
  const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
  std::mt19937_64 rng(20261018);
  std::printf("%s\n", cs_version());
  check_plan(rng, iters);
  check_planners(rng, iters);
  check_rejections();
  check_oracle(rng);
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host ABI checks passed (%d plan shapes)\n", iters);
  return 0;
}
