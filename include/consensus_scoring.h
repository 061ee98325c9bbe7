/*
 * consensus_scoring.h — C-ABI of the MI355X (gfx950) agent x candidate scoring path.
 *
 * The reference (cartgr/Generating-Fair-Consensus-Statements-with-Social-Choice-on-Token-Level-MDPs)
 * has no native code and no FFI: every log-probability comes back from a remote
 * HTTPS call (`get_prompt_logprobs`, src/utils.py:201-281) and is folded into
 * per-agent utilities and welfare by serial Python loops.  This header is the
 * boundary that replaces those loops.  Each entry point names the reference code
 * it replaces (file:line, relative to the reference root).
 *
 * Conventions
 *   - All data pointers are caller-owned DEVICE buffers (e.g. torch tensors'
 *     data_ptr()).  The library never allocates on the hot path; the only scratch
 *     is the caller-provided workspace sized by cs_workspace_size().
 *   - Every call is asynchronous and stream-ordered on `stream` (a hipStream_t
 *     passed as an opaque pointer; NULL = the default stream).  No host sync.
 *   - Return value: CS_OK (0) on success, a negative cs_status otherwise; the
 *     message is available from cs_last_error() (thread-local).
 *   - Kernels are re-entrant: no global mutable device state.
 *   - Results are deterministic run-to-run: no float atomics, fixed reduction order.
 */
#ifndef CONSENSUS_SCORING_H
#define CONSENSUS_SCORING_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* cs_stream_t; /* hipStream_t */

/* element type of the logits buffer */
enum cs_dtype { CS_F32 = 0, CS_BF16 = 1, CS_F16 = 2 };

/* welfare over agents (applied per candidate column) */
enum cs_welfare {
  CS_WELFARE_MIN = 0,    /* egalitarian: min_a u[a,c]                                  */
  CS_WELFARE_SUM = 1,    /* utilitarian: sum_a u[a,c]                                  */
  CS_WELFARE_SUMLOG = 2, /* log-Nash:    sum_a log(max(u[a,c], eps))                   */
  CS_WELFARE_MAX = 3     /* max_a u[a,c] (egalitarian over a cost, e.g. perplexity)    */
};

/* what cs_welfare_reduce does with a non-finite utility */
enum cs_nonfinite {
  CS_NONFINITE_SKIP = 0,   /* drop it (src/evaluation.py:316-319, `np.isfinite` filter)        */
  CS_NONFINITE_REPLACE = 1 /* nan_to_num(nan, posinf, neginf) (src/methods/best_of_n.py:384-389) */
};

enum cs_status {
  CS_OK = 0,
  CS_ERR_INVALID = -1,   /* bad argument (shape, dtype, null pointer)          */
  CS_ERR_WORKSPACE = -2, /* workspace missing or smaller than cs_workspace_size */
  CS_ERR_HIP = -3        /* a HIP launch failed                                 */
};

/* Library identification and last error (thread-local, never NULL). */
const char* cs_version(void);
const char* cs_last_error(void);

/* Bytes of device workspace cs_logsoftmax_gather needs for this shape (0 when the
 * single-pass path is used).  Pure host function. */
size_t cs_workspace_size(int64_t rows, int64_t vocab, int32_t k);

/*
 * cs_logsoftmax_gather — fused vocab-wide log-softmax + candidate-token gather.
 *
 * For every row r of logits[rows][ld] (first `vocab` columns used):
 *     x'       = softcap > 0 ? softcap * tanh(x / softcap) : x
 *     lse[r]   = log(sum_v exp(x'[r,v]))
 *     out_tok_lp[r*k + j] = x'[r, target_ids[r*k + j]] - lse[r]      (j < k)
 * A target id outside [0, vocab) yields NaN (the reference's `None` log-prob,
 * src/utils.py:262-263, which every caller filters).
 * One HBM pass over the logits; fp32 accumulation.
 *
 * Replaces: the remote log-softmax + gather behind get_prompt_logprobs
 *   (src/utils.py:249-263, echo=True prompt log-probs), the per-token read in
 *   _get_agent_token_logprob (src/methods/beam_search.py:389-390; one row per
 *   (agent, beam) gathered at k candidate tokens), and core.log_softmax_rows +
 *   gather (core.py:64-68, 88-90).
 *
 * out_row_lse may be NULL.  workspace may be NULL iff cs_workspace_size() == 0.
 */
int cs_logsoftmax_gather(const void* logits, int dtype, int64_t rows, int64_t vocab, int64_t ld,
                         const int32_t* target_ids, int32_t k, float softcap, float* out_tok_lp,
                         float* out_row_lse, void* workspace, size_t workspace_bytes,
                         cs_stream_t stream);

/*
 * cs_segment_reduce — per-candidate folding of token log-probs.
 *
 * Segment s covers tok_lp[seg_offsets[s] .. seg_offsets[s+1]) (CSR, non-decreasing).
 * NaN entries (None log-probs) are skipped.  Sums are accumulated in fp64 in a
 * fixed order.  Outputs (any may be NULL):
 *     out_sum_lp[s] = sum lp        out_sum_p[s] = sum exp(lp)
 *     out_count[s]  = #non-NaN      out_last[s]  = tok_lp[seg_offsets[s+1]-1] (NaN if empty)
 *
 * Replaces: mean of valid log-probs (src/methods/best_of_n.py:303-305),
 *   np.mean(logprobs[-len(path):]) (src/methods/finite_lookahead.py:508-520),
 *   avg_logprob / avg_prob (src/evaluation.py:203-213), sum(full_logprobs[-1:])
 *   (src/methods/beam_search.py:389-390), logu[:, j] += ls[:, a_t] (core.py:90).
 */
int cs_segment_reduce(const float* tok_lp, int64_t n, const int32_t* seg_offsets, int64_t n_seg,
                      float* out_sum_lp, float* out_sum_p, int32_t* out_count, float* out_last,
                      cs_stream_t stream);

/*
 * cs_welfare_reduce — welfare across agents for every candidate.
 *
 * U is [A][C] with row stride ldu (agent-major, agent order = dict order of
 * agent_opinions).  W[c] = welfare_kind over a of U[a*ldu + c], folded in agent
 * order in fp64.  Non-finite utilities are skipped or replaced (cs_nonfinite);
 * a column with no usable utility gives NaN.
 *
 * Replaces: min over agents (src/methods/beam_search.py:558-560,
 *   src/methods/best_of_n.py:401-408, src/methods/finite_lookahead.py:527);
 *   utilitarian / log-Nash welfare (src/evaluation.py:337-349, 367-381);
 *   F_val at a point-mass lottery (core.py:108-113); utilitarian column sums
 *   (core.py:374).
 */
int cs_welfare_reduce(const float* U, int32_t A, int32_t C, int64_t ldu, int kind, float eps,
                      int nonfinite, float nan_val, float posinf_val, float neginf_val, float* W,
                      cs_stream_t stream);

/*
 * cs_segmented_topk — stable descending top-k inside each segment.
 *
 * Segment s is W[s*ld .. s*ld + seg_len).  out_idx[s*k + r] is the index (within
 * the segment) of the element of rank r, ranks ordered by (value desc, index asc);
 * NaN ranks below every number.  out_val may be NULL.  k <= seg_len <= 16384.
 *
 * Replaces: sorted(candidates, key=min(rewards), reverse=True) — stable, so ties
 *   keep insertion order (src/methods/beam_search.py:558-560, 646-648);
 *   np.argmax, first max wins (src/methods/best_of_n.py:198, core.py:374);
 *   max(range, key=...) (src/methods/finite_lookahead.py:527).
 */
int cs_segmented_topk(const float* W, int32_t n_seg, int32_t seg_len, int64_t ld, int32_t k,
                      int32_t* out_idx, float* out_val, cs_stream_t stream);

/*
 * cs_beam_step — one scoring step of token-level beam search after the LM head, in ONE
 * launch (one workgroup per (agent row, vocab split); the last workgroup of each row
 * finishes that row, the last row folds the welfare and sorts).
 *
 * logits holds the agent rows [A*B][ld] (row a*B + b = agent a's prompt + beam b);
 * targets [B][K] are the candidate tokens of beam b, shared by every agent (an id
 * outside [0, vocab) is padding and yields NaN); rewards_in [A][B] is each agent's
 * cumulative reward of each beam.  With C = B*K and c = b*K + j:
 *     lp           = x'[a*B+b, targets[c]] - lse[a*B+b]           (as cs_logsoftmax_gather)
 *     out_U[a*C+c] = rewards_in[a*B+b] + lp                      (fp32 add)
 *     out_W[c]     = welfare_kind over a of out_U[a*C+c]         (as cs_welfare_reduce, SKIP)
 *     out_order[r] = index of rank r by (W desc, index asc), NaN last, r < n_order
 *                    (as cs_segmented_topk); out_order_val (nullable) = W at that index.
 *     out_kept[a*n_order + r] (nullable) = out_U[a*C + out_order[r]]: the cumulative
 *                    rewards of the kept beams when the first n_order ranks are kept
 *                    (needs n_order > 0 and B*K <= 1024).
 * n_order <= 256 selects the n_order best (radix-select threshold + rank counting, the
 * exact stable order) without sorting the rest.
 * Bit-identical to cs_logsoftmax_gather + cs_welfare_reduce + cs_segmented_topk on the
 * same inputs.  n_order = 0 skips the sort (agent-sharded runs all-reduce out_W
 * first, then call cs_segmented_topk).  B*K <= 16384 (a second launch sorts when
 * B*K > 1024).
 *
 * WORKSPACE: cs_beam_step_workspace_size() bytes, zero-filled before the first call and
 * used by one stream at a time.  It holds arrival counters that every call leaves at
 * zero, so it is reused without a memset (and inside captured graphs).
 *
 * Replaces: the per-(beam, token, agent) scoring loop, cumulative rewards and the
 *   stable sort by min over agents of src/methods/beam_search.py:495-560
 *   (_get_agent_token_logprob :335-404 per candidate).
 */
size_t cs_beam_step_workspace_size(int64_t rows, int64_t vocab);
int cs_beam_step(const void* logits, int dtype, int32_t A, int32_t B, int64_t vocab, int64_t ld,
                 const int32_t* targets, int32_t K, const float* rewards_in, float softcap,
                 int welfare_kind, float eps, float* out_U, float* out_W, int32_t n_order,
                 int32_t* out_order, float* out_order_val, float* out_kept, void* workspace,
                 size_t workspace_bytes, cs_stream_t stream);

/*
 * cs_beam_decode_step — one whole beam-search decode step after the LM head in ONE
 * launch: cs_vocab_topk on the B reference-policy rows (ref_logits [B][ld_ref]) proposes
 * K candidate tokens per beam (out_ids [B][K], value desc / id asc), and cs_beam_step
 * scores them under the agent rows (logits [A*B][ld]) — out_U, out_W, out_order,
 * out_order_val, out_kept exactly as cs_beam_step with targets = out_ids.  The proposer
 * workgroups run beside the agent-row stream; per beam the last of its A + 1 arrivals
 * gathers the beam's candidates.  Bit-identical to cs_vocab_topk + cs_beam_step.
 * Limits: K <= min(256, vocab), B*K <= 16384, A*B <= 65536, B <= 4096.
 *
 * WORKSPACE: cs_beam_decode_workspace_size() bytes, zero-filled before the first call,
 * used by one stream at a time, left zeroed by every call (graph-replayable).
 *
 * Replaces: the reference's per-step loop of beam_search.py:439-560 — unique-token
 *   sampling per beam (:199-333), per (beam, token, agent) scoring (:335-404, 495-538),
 *   cumulative rewards and the stable sort by min over agents (:534-560).
 */
size_t cs_beam_decode_workspace_size(int32_t A, int32_t B, int64_t vocab, int32_t K);
int cs_beam_decode_step(const void* ref_logits, int64_t ld_ref, const void* logits, int64_t ld,
                        int dtype, int32_t A, int32_t B, int64_t vocab, int32_t K, float softcap,
                        const float* rewards_in, int welfare_kind, float eps, int32_t* out_ids,
                        float* out_U, float* out_W, int32_t n_order, int32_t* out_order,
                        float* out_order_val, float* out_kept, void* workspace,
                        size_t workspace_bytes, cs_stream_t stream);

/*
 * cs_beam_select — the selection half of an agent-sharded beam step, after the welfare
 * all-reduce: out_order[r] = index of rank r of W by (W desc, index asc), NaN last,
 * r < n_order (as cs_segmented_topk); out_order_val (nullable) = W there; out_kept
 * (nullable) [A][n_order] = U[a*C + out_order[r]] for this rank's A agents (U [A][C],
 * the out_U of its cs_beam_decode_step / cs_beam_step); out_W (nullable) = W after
 * unfill.  unfill: CS_UNFILL_POSINF turns +inf back into NaN (the MIN combine fills
 * columns without a usable utility with +inf before the all-reduce, parallel.py),
 * CS_UNFILL_NEGINF does the same for -inf (MAX), CS_UNFILL_NONE leaves W as is.
 * One workgroup, one launch; C <= 1024, 0 < n_order <= C.  Bit-identical to
 * cs_segmented_topk + the column gather.
 *
 * Replaces: the stable sort by min over agents and the keep of the first beam_width of
 *   src/methods/beam_search.py:558-593 on a rank that holds a subset of the agents.
 */
#define CS_UNFILL_NONE 0
#define CS_UNFILL_POSINF 1
#define CS_UNFILL_NEGINF 2
int cs_beam_select(const float* W, int32_t C, int unfill, const float* U, int32_t A,
                   int32_t n_order, float* out_W, int32_t* out_order, float* out_order_val,
                   float* out_kept, cs_stream_t stream);

/*
 * cs_vocab_topk — deterministic candidate proposer: the k largest (soft-capped)
 * logits of every row, ordered by (value desc, token id asc).
 *
 * Replaces the serial unique-token sampling loop of the reference's beam search
 * (_sample_next_tokens, src/methods/beam_search.py:199-333: up to
 * max_sampling_attempts remote completions per beam) with one HBM pass per step;
 * k is the build's deterministic "top-k tokens per beam" (BASELINE configs).
 * Logit-bias masking (beam_search.py:236-251) is applied by the caller to the
 * logits rows before the call.  k <= 256 and ceil(vocab/4096)*k <= 16384.
 * out_vals may be NULL.
 */
size_t cs_vocab_topk_workspace_size(int64_t rows, int64_t vocab, int32_t k);
int cs_vocab_topk(const void* logits, int dtype, int64_t rows, int64_t vocab, int64_t ld, int32_t k,
                  float softcap, int32_t* out_ids, float* out_vals, void* workspace,
                  size_t workspace_bytes, cs_stream_t stream);

/*
 * cs_vocab_sample — seeded Gumbel-max sampling, n_draw independent draws per row.
 *
 * Draw d of row r returns argmax_v ( x'[r,v] / temperature + g(seeds[r*n_draw+d], v) ),
 * ties to the lowest id, with g = -log(-log(u)) and u the counter-based uniform
 * documented in oracle/oracle.py (splitmix64 of (seed, v), top 23 bits + 0.5, scaled by 2^-23).
 * out_lp (nullable) receives the drawn token's log-probability under
 * softmax(x'/temperature).  n_draw <= 16.
 *
 * Replaces the remote one-token samplers: client.completions.create(max_tokens=1,
 * seed=base_seed+attempt, logit_bias) (src/methods/beam_search.py:253-297),
 * generate_text(max_tokens=1, temperature=1, seed) in the lookahead tree
 * (src/methods/finite_lookahead.py:310-334) and the per-token draws of the
 * Best-of-N candidate generation (src/methods/best_of_n.py:104-118).
 */
size_t cs_vocab_sample_workspace_size(int64_t rows, int64_t vocab, int32_t n_draw);
int cs_vocab_sample(const void* logits, int dtype, int64_t rows, int64_t vocab, int64_t ld,
                    float temperature, float softcap, const uint64_t* seeds, int32_t n_draw,
                    int32_t* out_ids, float* out_lp, void* workspace, size_t workspace_bytes,
                    cs_stream_t stream);

/*
 * cs_prefix_attention — cascade attention of many candidate streams over SHARED
 * per-agent prefix K/V (bf16 in / bf16 out, fp32 online softmax, bf16 MFMA).
 *
 * n_groups groups of n_str streams each; group i uses prefix group_prefix[i] (NULL =
 * identity).  Stream s = i*n_str + b carries T query tokens; token t of stream s is
 * q[(s*T + t)][H][D] and sees
 *     prefix keys  [0, prefix_len[pfx])   k_prefix  [Hkv][ld_prefix][D]
 *                                         vt_prefix [Hkv][ld_prefix/32][D][32]
 *                                         prefix p's key j is row prefix_off[p] + j (ragged
 *                                         prefixes in one buffer; prefix_off[p] % 32 == 0,
 *                                         rows up to the next multiple of 32 readable)
 *     its history  [0, *hist_base + t]    k_hist  [S][Hkv][ld_hist][D]
 *                                         vt_hist [S][Hkv][ld_hist/32][D][32]
 * V is stored transposed in 32-key tiles: keys 32c .. 32c+31 are the tile
 * vt[..][c][0..D)[0..32), key-contiguous rows of 64 B.  ld_prefix, ld_hist multiples of 32;
 * key slots past the visible range must hold finite values.  out [(s*T + t)][H][D].
 * Query head h uses K/V head h / (H / Hkv).  scores = q.k * scale, then
 * softcap * tanh(./softcap) when softcap > 0 (Gemma-2 attention soft-cap), softmax over the
 * visible keys; window > 0 also hides keys more than window - 1 positions behind the query
 * (Gemma-2's sliding window; prefix key j sits at position j, history slot j at
 * prefix_len + j).  D in {64, 128, 256}.  hist_base lives in device memory so that a
 * captured decode step replays with a growing history.  max_prefix_len (host) bounds
 * prefix_len.  One workgroup holds all query rows of (group, K/V head) (64 per workgroup),
 * so a prefix key block is read once for every candidate of that agent.
 *
 * Work plan: when few (group, head, query group) cells would leave the chip idle (decode
 * steps), each cell's keys are split over several workgroups and the splits merged in a
 * second launch.  cs_prefix_attention_plan (host) sizes the splits per cell from host
 * bounds of the prefix lengths (prefix_len[p] >= the device length; the split count is a
 * performance choice only) and the history capacity, and writes int32 x 4 entries:
 *     plan == NULL:  returns the entry count (0 = no plan needed: pass plan = NULL, no
 *                    workspace), n_attn / n_merge / workspace_bytes through the pointers;
 *     plan != NULL:  fills up to plan_cap entries.
 * The caller copies the entries to device memory once per prefix set and passes them with
 * n_attn, n_merge and a workspace of workspace_bytes.  Results are deterministic (fixed-order
 * split merge), and equal for every plan up to fp32 reassociation.
 *
 * Replaces: the per-(agent, candidate) re-encoding of the agent's whole prompt behind
 *   every get_prompt_logprobs call (src/utils.py:249-259; driven per candidate at
 *   src/methods/beam_search.py:495-538, best_of_n.py:266-321,
 *   finite_lookahead.py:464-524, src/evaluation.py:177-230).
 */
int64_t cs_prefix_attention_plan(const int32_t* prefix_len, int32_t n_prefix,
                                 const int32_t* group_prefix, int32_t n_groups, int32_t n_str,
                                 int32_t T, int32_t H, int32_t Hkv, int32_t D, int64_t ld_hist,
                                 int32_t* plan, int64_t plan_cap, int32_t* n_attn, int32_t* n_merge,
                                 size_t* workspace_bytes);
int cs_prefix_attention(const void* q, const void* k_prefix, const void* vt_prefix,
                        int64_t ld_prefix, const int64_t* prefix_off, const int32_t* prefix_len,
                        int32_t max_prefix_len, const int32_t* group_prefix, int32_t n_groups,
                        const void* k_hist, const void* vt_hist, int64_t ld_hist,
                        const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H, int32_t Hkv,
                        int32_t D, float scale, float softcap, int32_t window, const void* plan,
                        int32_t n_attn, int32_t n_merge, void* out, void* workspace,
                        size_t workspace_bytes, cs_stream_t stream);

/*
 * cs_prefix_attention_rows — cs_prefix_attention over a ROW-LAYOUT history reached through a
 * slot table, for beam decoding without history copies:
 *     k_hist, v_hist  [S][Hkv][ld_hist][D] (V row-major like K, not in 32-key V^T tiles)
 *     hist_rows       [S][ld_hist] int32: slot j of stream s is row hist_rows[s][j] of k_hist /
 *                     v_hist (every entry a row of the buffers, which may hold more than the
 *                     S query streams: a token tree's earlier levels)
 * so a beam's inherited slots stay where its ancestor wrote them (cs_hist_rows_update builds
 * the next step's table; cs_rope_place_rows writes the step's K / V into the stream's own row).
 * Same arguments, plan and results otherwise (plan may be NULL with no workspace: one
 * workgroup per (group, K/V head, query group)).  Every result equals cs_prefix_attention on
 * the copied history the table describes, up to fp32 reassociation (the same block order:
 * bitwise in practice).
 *
 * Replaces: as cs_prefix_attention; the beam's history is the reference's beam text
 *   (src/methods/beam_search.py:491-538), re-encoded in full by every call there.
 */
int cs_prefix_attention_rows(const void* q, const void* k_prefix, const void* vt_prefix,
                             int64_t ld_prefix, const int64_t* prefix_off, const int32_t* prefix_len,
                             int32_t max_prefix_len, const int32_t* group_prefix, int32_t n_groups,
                             const void* k_hist, const void* v_hist, const int32_t* hist_rows,
                             int64_t ld_hist, const int32_t* hist_base, int32_t n_str, int32_t T,
                             int32_t H, int32_t Hkv, int32_t D, float scale, float softcap,
                             int32_t window, const void* plan, int32_t n_attn, int32_t n_merge,
                             void* out, void* workspace, size_t workspace_bytes, cs_stream_t stream);

/*
 * cs_rope_place — rotary embedding (half-rotation convention, angle = position *
 * inv_freq[i]) of the fused projection qkv [(s*T + t)][ld_qkv] = [q (H*D) | k (Hkv*D) |
 * v (Hkv*D)] and placement into the cs_prefix_attention layouts: q_out [(s*T+t)][H][D],
 * k_hist[s][g][j][:] (rotated), vt_hist[s][g][j/32][:][j%32], j = *hist_base + t.  The
 * position of token t of stream s (group i) is prefix_len[group_prefix[i]] + *hist_base + t.
 * bf16 in / out, fp32 rotation.
 *
 * Replaces: the per-call re-encoding of the reference's prompts (src/utils.py:249-259):
 *   a candidate token's K/V is computed once and kept for every later step of its stream.
 */
int cs_rope_place(const void* qkv, int64_t ld_qkv, const float* inv_freq, const int32_t* prefix_len,
                  const int32_t* group_prefix, int32_t n_groups, const int32_t* hist_base,
                  int32_t n_str, int32_t T, int32_t H, int32_t Hkv, int32_t D, void* q_out,
                  void* k_hist, void* vt_hist, int64_t ld_hist, cs_stream_t stream);

/*
 * cs_rope_place_splitk — cs_rope_place on a K-split projection's unfolded fp32 partials
 * part [splits][n_tok][(H + 2 Hkv) D] (cs_gemm_bf16 with y = NULL): each element is summed in
 * split order and rounded to bf16 exactly as cs_gemm_bf16's own fold would, then rotated and
 * placed -- bitwise cs_gemm_bf16 (folded) followed by cs_rope_place, one launch fewer.
 * T < 32, head_dim % 16 == 0, part 16-byte aligned.
 *
 * Replaces: as cs_rope_place (src/utils.py:249-259).
 */
int cs_rope_place_splitk(const float* part, int32_t splits, const float* inv_freq,
                         const int32_t* prefix_len, const int32_t* group_prefix, int32_t n_groups,
                         const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H,
                         int32_t Hkv, int32_t D, void* q_out, void* k_hist, void* vt_hist,
                         int64_t ld_hist, cs_stream_t stream);

/*
 * cs_rope_place_rows / cs_rope_place_splitk_rows — cs_rope_place / cs_rope_place_splitk with
 * V placed row-major like K: v_hist[s][g][j][:] (the cs_prefix_attention_rows layout), in the
 * stream's own row s.
 *
 * Replaces: as cs_rope_place (src/utils.py:249-259).
 */
int cs_rope_place_rows(const void* qkv, int64_t ld_qkv, const float* inv_freq,
                       const int32_t* prefix_len, const int32_t* group_prefix, int32_t n_groups,
                       const int32_t* hist_base, int32_t n_str, int32_t T, int32_t H, int32_t Hkv,
                       int32_t D, void* q_out, void* k_hist, void* v_hist, int64_t ld_hist,
                       cs_stream_t stream);
int cs_rope_place_splitk_rows(const float* part, int32_t splits, const float* inv_freq,
                              const int32_t* prefix_len, const int32_t* group_prefix,
                              int32_t n_groups, const int32_t* hist_base, int32_t n_str, int32_t T,
                              int32_t H, int32_t Hkv, int32_t D, void* q_out, void* k_hist,
                              void* v_hist, int64_t ld_hist, cs_stream_t stream);

/*
 * cs_hist_rows_update — the beam (or token-tree) step of a row-layout history
 * (cs_prefix_attention_rows):
 *     dst_rows[s][j] = src_rows[parent[s]][j]   j < *hist_base   (inherited slots, by table)
 *     dst_rows[s][j] = row_base + s             j >= *hist_base  (written by this and later steps)
 * dst [S][ld_hist] int32; src [any][ld_hist] (the parents' table: the previous beam step's,
 * or a token tree's parent level's), distinct from dst.  Beams: one buffer of S rows,
 * row_base 0, a ping-pong pair of tables so a queued step can be undone; a token tree: one
 * buffer for every level's streams, a level's streams at rows row_base .. row_base + S - 1.
 * n_rows: the K / V buffer's row count; row_base + S > n_rows is rejected (CS_ERR_INVALID),
 * so a table can never name a row past the buffer it indexes.  No K / V moves.  hist_base
 * in device memory (graph replays).
 *
 * Replaces: the reference's beams and lookahead paths are strings that every scoring call
 *   re-encodes in full (src/methods/beam_search.py:491-538, src/methods/finite_lookahead.py:
 *   297-399 through src/utils.py:249-259); here a kept beam or a tree node inherits its
 *   parent's K / V by table, without any copy.
 */
int cs_hist_rows_update(const int32_t* src_rows, int32_t* dst_rows, const int64_t* parent,
                        const int32_t* hist_base, int64_t S, int32_t ld_hist, int64_t row_base,
                        int64_t n_rows, cs_stream_t stream);

/*
 * cs_add_rms_norm — residual add + RMSNorm of bf16 rows in one pass:
 *     b' = b, or with b_weight: b' = b * rsqrt(mean(b^2) + eps) * g_b (rounded to bf16; the
 *          branch's own norm, Gemma-2's post-attention / post-MLP norm, bitwise as a
 *          separate cs_add_rms_norm over b alone)
 *     s = a + b' (rounded to bf16; b NULL = none), written to s_out when non-NULL (may alias a)
 *     y = s * rsqrt(mean(s^2) + eps) * g,  g = weight (plus_one = 0, Llama-3) or
 *         1 + weight (plus_one = 1, Gemma-2; also g_b); fp32 statistics, one rounding.
 * d a multiple of 8 (<= 32768), leading dimensions multiples of 8.
 *
 * Replaces: part of the remote forward behind every get_prompt_logprobs call
 *   (src/utils.py:249-259) — the per-layer residual + normalisation of each new token.
 */
int cs_add_rms_norm(const void* a, int64_t lda, const void* b, int64_t ldb, const void* b_weight,
                    void* s_out, int64_t lds, const void* weight, int64_t rows, int64_t d,
                    float eps, int plus_one, void* y, int64_t ldy, cs_stream_t stream);

/*
 * cs_add_rms_norm_splitk — cs_add_rms_norm whose branch b is the K-split partials of a
 * cs_gemm_bf16 called with y = NULL: partials [splits][rows][d] fp32 (contiguous, 16-byte
 * aligned, 1 <= splits <= 16, d <= 8192) are folded in split order and rounded to bf16 exactly as cs_gemm_bf16's own fold,
 * so the result is bitwise cs_gemm_bf16(y) followed by cs_add_rms_norm(b = y) — one launch
 * and one bf16 round trip fewer (a decode step's down projection + the residual add).
 */
int cs_add_rms_norm_splitk(const void* a, int64_t lda, const float* partials, int32_t splits,
                           const void* b_weight, void* s_out, int64_t lds, const void* weight,
                           int64_t rows, int64_t d, float eps, int plus_one, void* y, int64_t ldy,
                           cs_stream_t stream);

/*
 * cs_gated_act — the gated MLP activation of bf16 rows: out = act(gate) * up with act =
 * SiLU (act = 0, Llama-3) or tanh-GeLU (act = 1, Gemma-2), the activation rounded to bf16
 * before the product.  F and leading dimensions multiples of 8.
 *
 * Replaces: part of the remote forward behind every get_prompt_logprobs call
 *   (src/utils.py:249-259).
 */
int cs_gated_act(const void* gate, int64_t ld_gate, const void* up, int64_t ld_up, int64_t rows,
                 int64_t F, int act, void* out, int64_t ld_out, cs_stream_t stream);

/*
 * cs_gemm_bf16 — a decode step's projection GEMM, Y[M, N] = X[M, K] * W[N, K]^T, bf16 in
 * and out, fp32 accumulation (v_mfma_f32_16x16x32_bf16), for the few hundred rows one step
 * of all (agent, beam) streams has.  W (the streamed operand, read once) is [N, K] row-major
 * (a torch Linear weight); X [M, K]; Y [M, N] (gated = 0).  gated = 1: W is the fused
 * gate|up weight [2F, K] (gate rows first) and Y [M, F] = act(gate) * up with the rounding
 * of cs_gated_act (act 0 SiLU, 1 tanh-GeLU).  splits > 1 divides K over workgroups and
 * folds the fp32 partials in split order (workspace: splits * M * N floats); splits <= 0
 * takes cs_gemm_splits; y = NULL with splits > 1 leaves the partials [splits][M][N] in the
 * workspace unfolded (cs_add_rms_norm_splitk folds them).  variant: 0 = the library's choice, 1 = 2 x 4 wave grid (128 columns x
 * up to 288 rows per workgroup), 2 = column-only wave split, 256 columns, LDS-DMA X,
 * 3 = as 2 with 128 columns (gated: 4 waves, 64 features per workgroup, two workgroups per
 * CU; N a multiple of 128), 4 = as 2 with at most 144 rows per workgroup (row blocks of a
 * column tile paired on one XCD); 5-7 = the thin form for M <= 80 (no K split: every wave
 * of a workgroup streams its own K slice into registers, no barrier until the final fold;
 * 5: 16 features x 8 waves, 6: 32 x 8, 7: 16 x 16).  N a multiple of 128, K of 64 * splits;
 * ldx, ldw multiples of 8, ldy of 4; X, W 16-byte aligned.  Deterministic (no atomics).
 *
 * Replaces: part of the remote forward behind every get_prompt_logprobs call
 *   (src/utils.py:249-259) — the per-layer q|k|v, output, gate|up and down projections of
 *   each new token (the gated form also replaces cs_gated_act on that path).
 */
int cs_gemm_bf16(const void* x, int64_t ldx, const void* w, int64_t ldw, void* y, int64_t ldy,
                 int64_t M, int64_t N, int64_t K, int splits, int gated, int act, int variant,
                 float* workspace, cs_stream_t stream);

/* cs_gemm_splits — the K split cs_gemm_bf16 takes for splits <= 0 (>= 1; 0 on a bad shape). */
int64_t cs_gemm_splits(int64_t M, int64_t N, int64_t K, int gated, int variant);

/*
 * cs_gemm_pack — W [N, K] (row stride ldw) into the fragment-major layout of
 * cs_gemm_bf16_packed: 16-row tile T, 64-deep K step s, half h (k 32h .. 32h + 31) is 1 KB at
 * element ((T * K / 64 + s) * 2 + h) * 512, lane-linear (lane l's 8 elements = row 16T + l % 16,
 * k 64s + 32h + 8 (l / 16) .. + 7).  A pure permutation (N * K elements out); N % 16 == 0,
 * K % 64 == 0, 16-byte aligned.  Done once per weight, at model load.
 *
 * cs_gemm_bf16_packed — cs_gemm_bf16 (variants 0, 2, 3, 4; same splits, gated, act, workspace
 * rules) on a packed W: every weight-fragment load is one contiguous 1 KB and each wave's W
 * stream one sequential run, instead of 16 rows x 64 B.  Bitwise equal to cs_gemm_bf16 on the
 * unpacked W.
 *
 * Replaces: the same projections of the remote forward as cs_gemm_bf16
 *   (src/utils.py:249-259).
 */
int cs_gemm_pack(const void* w, int64_t ldw, int64_t N, int64_t K, void* w_packed,
                 cs_stream_t stream);

int cs_gemm_bf16_packed(const void* x, int64_t ldx, const void* w_packed, void* y, int64_t ldy,
                        int64_t M, int64_t N, int64_t K, int splits, int gated, int act,
                        int variant, float* workspace, cs_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* CONSENSUS_SCORING_H */
