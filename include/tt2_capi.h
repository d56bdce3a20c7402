/* tt2_capi.h -- C ABI of libtt2.so, the MI355X (gfx950) kernel library behind the
 * Transformer-TTS mel path (encoder -> decoder -> post-net).
 *
 * The reference (keonlee9420/Transformer-tacotron2, /root/reference/README.md:1-3)
 * ships no code, so it has no FFI to mirror; this ABI is the boundary SURVEY.md
 * section 8(b) defines: one entry point per fused block of the path, plain
 * pointers and sizes, no torch types.  INTEGRATION.md shows the ctypes binding.
 *
 * Conventions
 *  - Every device buffer (inputs, outputs, workspace) is allocated by the caller;
 *    nothing allocates on the hot path, so every call is hipGraph-capturable.
 *  - Calls are stream-ordered on the caller's stream and reentrant.
 *  - Return 0 (TT2_OK) or a negative TT2_E_* code; tt2_last_error() returns a
 *    thread-local message for the last failure on this thread.
 *  - dtype fields: TT2_DT_F32 = 0, TT2_DT_BF16 = 1, TT2_DT_F16 = 2 (decode step only).  Activations are
 *    channels-last row-major [rows, channels]; rows = batch * time.
 *  - Dropout: keep(idx) = hash(seed, site, idx) >= thr; thr = 0
 *    disables it.  seed points to a device uint32.
 */
#ifndef TT2_CAPI_H
#define TT2_CAPI_H
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TT2_OK 0
#define TT2_E_INVALID -1
#define TT2_E_LAUNCH -2
#define TT2_E_HIP -3

#define TT2_DT_F32 0
#define TT2_DT_BF16 1
#define TT2_DT_F16 2   /* decode step only: skinny GEMM, decode attention, ln_combine, cast2d */

/* ------------------------------------------------------------------ runtime */
const char* tt2_last_error(void);
int tt2_version(void);
int tt2_init(int device);

/* --------------------------------------------------------------------- GEMM
 * C[m,n] = epi(alpha * sum_k A(m,k) B(n,k)), epi = (+bias[n]) (+res[m,n]) (act)
 *          (*gate: res==0 ? 0 : gate_scale) (dropout) (+beta*C[m,n]).
 * trans_a = 0: A(m,k) = a[m*lda + k]; 1: a[k*lda + m].  trans_b likewise for B(n,k).
 * a_conv_t > 0: A is the implicit im2col of a channels-last sequence batch
 *   (time = m % a_conv_t, tap = k / a_conv_c, zero outside [0, T)); b_conv_* the
 *   same for an N-contiguous B (wgrad of a conv).
 * splits > 1: split-K with an f32 workspace of tt2_gemm_workspace_size() bytes.
 * Replaces the nn.Linear / nn.Conv1d products of SURVEY 8(a) rows a1, a3-a9, a11. */
typedef struct tt2_gemm_args {
  const void* a; const void* b; void* c;
  const float* bias;
  const void* res; const void* gate;
  const uint32_t* drop_seed;
  void* workspace; size_t ws_bytes;
  int64_t lda, ldb, ldc, ldr, ldg;
  int32_t m, n, k;
  int32_t dtype_in, dtype_out, res_dtype, gate_dtype;
  int32_t trans_a, trans_b;
  int32_t act;          /* 0 none, 1 relu, 2 tanh */
  int32_t splits;
  float alpha, beta, gate_scale;
  uint32_t drop_site, drop_thr;
  float drop_scale;
  int32_t a_conv_t, a_conv_c, a_conv_pad;
  int32_t b_conv_t, b_conv_c, b_conv_pad;
  int32_t kernel_variant;  /* 0 auto, 1 register-staged (any shape), 2 LDS-DMA 128x128 (bf16, 8-aligned inner
                              dims), 13 / 14 warp-specialised 256x128 (same, conv C, T >= 64; the auto choice
                              when eligible) with its register / LDS-image epilogue (auto: LDS image),
                              15 64x64 (K-contiguous A; auto for <= 64 v7 tiles), 16 256x256 (NT, bf16 C,
                              N % 256 == 0, K % 64 == 0, bias / ReLU / dropout epilogues only; auto when
                              its rounds of the chip cost less than v7's), 17 256x128 with 8 loader waves
                              (NT, bf16 C, N % 128 == 0, K % 64 == 0, the same epilogues; auto where v7 would
                              run) */
  /* optional fused row sums of op(A) over k: a_ksum[m] = a_ksum_beta * a_ksum[m] + sum_k A(m, k)
   * (f32).  With A = dY^T of a weight-gradient GEMM this is the bias gradient, taken from the
   * A tiles already staged in LDS.  Requires bf16, trans_a, no conv on A. */
  float* a_ksum;
  float a_ksum_beta;
  /* decode-step fusions, skinny path only (bf16, m <= 64 (LN prologue m <= 32), A and B K-contiguous):
   * - LayerNorm prologue on A: when a_ln_gamma != NULL the GEMM multiplies
   *   h = LN(A + a_ln_branch) (row-wise over the k = 512 columns, eps a_ln_eps) instead of A,
   *   and writes h to a_ln_out [m, k] (ld k);
   * - KV-cache scatter epilogue: when kv_cache != NULL, output columns n >= kv_col0 are also
   *   stored to kv_cache[m * kv_bstride + (*kv_t) * kv_ld + (n - kv_col0)] (bf16). */
  const void* a_ln_branch;
  const float* a_ln_gamma;
  const float* a_ln_beta;
  void* a_ln_out;
  float a_ln_eps;
  void* kv_cache;
  const int32_t* kv_t;
  int32_t kv_col0;
  int64_t kv_bstride, kv_ld;
  /* measurement hook: with splits > 1, launch only the main kernel (partials stay in
   * the workspace, C is not written), so a per-kernel timing excludes the reduce */
  int32_t main_only;
  /* more decode-step epilogues, skinny path only:
   * - scaled positional encoding: when pe_table != NULL, out[m, n] += (*pe_alpha) *
   *   pe_table[(*pe_t) * n_cols + n] after the rest of the epilogue (f32 table [T][n]);
   * - frame emit (the mel/stop heads GEMM): when emit_mel != NULL, with t = *emit_t < emit_tmax,
   *   columns n < emit_nmels also go to emit_mel[(m * emit_tmax + t) * emit_nmels + n] (f32) and
   *   emit_prev[m * emit_nmels + n] (bf16, the next step's pre-net input), column emit_nmels to
   *   emit_stop[m * emit_tmax + t]; the last workgroup to finish then sets *emit_t = t + 1,
   *   *emit_seed += 1 (if non-NULL) and re-zeroes *emit_done (a device int the caller zeroes
   *   once).  Replaces the tt2_decode_emit launch. */
  const float* pe_table;
  const float* pe_alpha;
  const int32_t* pe_t;
  float* emit_mel;
  float* emit_stop;
  void* emit_prev;
  int32_t* emit_t;
  uint32_t* emit_seed;
  int32_t* emit_done;
  int32_t emit_nmels, emit_tmax;
  /* frame emit, stop handling: emit_stop_bias (optional f32 [m][emit_tmax]) is added to the stop
   * logit before it is stored (per-utterance length injection); emit_stop_len (optional int32 [m])
   * records t + 1 at the first frame whose stop logit >= emit_stop_thr (entries the caller set to
   * INT32_MAX mean "still running"). */
  const float* emit_stop_bias;
  int32_t* emit_stop_len;
  float emit_stop_thr;
  /* fused BatchNorm statistics: when col_stats != NULL, each 256-row chunk r of the stored
   * (bf16) output C also leaves its column moments, col_stats[(2 r) * n + j] = mean and
   * col_stats[(2 r + 1) * n + j] = sum over the chunk's rows of (C - mean)^2 (rows < m only),
   * in the chunk layout tt2_batchnorm_fwd reads with stats_rows = the chunk's rows.  A chunk is the
   * kernel's tile height, tt2_gemm_stats_rows(): 64 rows on the 64 x 64 kernel (plan 15), else 256
   * on the 256 x 128 LDS-image path (bf16 C, A and B K-contiguous, n % 128 == 0); bf16 C, 16-B
   * aligned rows and no split-K either way.  Other requests fail with TT2_E_INVALID. */
  float* col_stats;
  /* fused BatchNorm backward sums: when bn_bwd != NULL, C is that BatchNorm's dout (the gradient
   * of its output: bn_bwd->y is its input, mean / rstd / gamma / beta / act / dropout as for
   * tt2_batchnorm_bwd, c == n, m == m), and each 256-row chunk r of the stored (bf16) C leaves the
   * column sums of dpre = dout * keep * act'(z) and of dpre * xhat in bn_bwd->workspace
   * ([r][2][n], the layout tt2_batchnorm_bwd reads with stats_rows = tt2_gemm_stats_rows()).  The
   * tt2_bn_args struct is read during the call only.  Same path restrictions as col_stats. */
  const struct tt2_bn_args* bn_bwd;
} tt2_gemm_args;
#define TT2_GEMM_STATS_ROWS 256   /* the 256 x 128 kernel's chunk (tt2_gemm_stats_rows) */

size_t tt2_gemm_workspace_size(const tt2_gemm_args* a);
/* Rows per chunk of a col_stats / bn_bwd request's statistics (the kernel's tile height): 64 on
 * the 64 x 64 kernel, 256 on the 256 x 128 one, 0 when the request cannot fuse them.  Host-only. */
int32_t tt2_gemm_stats_rows(const tt2_gemm_args* a);
int tt2_gemm(const tt2_gemm_args* a, hipStream_t stream);
/* Kernel tt2_gemm would launch for these args (no device work): 1 register-staged
 * 128x128 (any dtype), 2 LDS-DMA 128x128 (bf16), 3 skinny decode (m <= 64),
 * 13 warp-specialised 256x128, 15 64x64; -1 invalid. */
int tt2_gemm_plan(const tt2_gemm_args* a);

/* Grouped GEMM: up to 8 independent problems in ONE launch of the v7 kernel (every
 * problem must be v7-eligible -- tt2_gemm_plan(p) == 13 -- and share trans_a/trans_b;
 * each problem's own splits / workspace; one grouped split-K reduce follows).  Used for
 * the weight gradients of a layer, which share K = tokens.  Replaces the per-linear
 * weight-gradient calls of the reference's autograd backward (see tt2_gemm). */
int tt2_gemm_grouped(const tt2_gemm_args* probs, int32_t n, hipStream_t stream);

/* Measurement probe (bench.py's live roofline): tt2_probe_arm() makes the next main GEMM
 * kernel (v7 / grouped v7 / v8 / LDS-DMA 128x128) launched on this thread by the NEXT
 * tt2_gemm / tt2_gemm_grouped call record its timing and returns the slot.  Eager: start /
 * stop events ride in the kernel's own dispatch (its execution, as rocprofv3 reports it),
 * read by tt2_probe_ms (-1 if no probe-capable kernel consumed the slot, or under capture).
 * Eager and under stream capture alike, v7 / v8 kernels also record their own span on the
 * device wall clock (tt2_probe_span_ms); nothing is added to a captured graph, so each
 * replay of it re-times the launch inside the replayed step.  Any path of that call
 * disarms the probe; tt2_probe_reset() frees every slot. */
int tt2_probe_arm(void);
float tt2_probe_ms(int slot);
/* The same launch's span as the kernel records it on the device wall clock (first workgroup
 * start to last wave end, no stream event around it): ms, -1 if unavailable.  Reading
 * re-arms the slot's record, so a graph replayed again records afresh. */
float tt2_probe_span_ms(int slot);
/* The raw span record of a slot (measurement tools): per work group {start, end} on the device
 * wall clock (hipDeviceAttributeWallClockRate kHz), copied to out[2 * groups]; returns the
 * number of work groups, -groups - 1 if cap is too small, -1 if the slot has no record.  Read
 * it before tt2_probe_span_ms, which clears the record. */
int tt2_probe_span_records(int slot, unsigned long long* out, int cap);
/* u64 slots per work group in tt2_probe_span_records' output: 2 ({start, end}); 32 in the
 * in-step GEMM phase build (-DTT2_PHASE=1, tools/g7_phases.py: s_memtime stamps of the K
 * steps and the epilogue after the pair). */
int tt2_probe_span_width(void);
void tt2_probe_reset(void);

/* ---------------------------------------------------------------- attention
 * Scaled dot-product attention over heads of width 64, read in place from
 * projection outputs: head h of row (b, t) of Q is q[(b*tq + t)*q_ld + 64h].
 * Key j of batch b is visible iff j < key_len[b] (key_len may be NULL) and,
 * if causal, j <= t.  A row with no visible key outputs 0.
 * lse: [batch*heads, tq] f32, log2-domain log-sum-exp of scale*log2(e)*QK^T
 * (+inf for empty rows); written by fwd, read by bwd.
 * bwd: delta [batch*heads, tq] f32 scratch; dq/dk/dv may alias column slices
 * of one fused gradient buffer.  Replaces SURVEY 8(a) a3, a6, a7 (+ a11). */
typedef struct tt2_attn_args {
  const void* q; const void* k; const void* v;
  const void* o;      /* bwd: forward output */
  const void* dout;   /* bwd: gradient of the output */
  void* o_out;        /* fwd: output */
  void* dq; void* dk; void* dv;
  float* lse; float* delta;
  int64_t q_ld, k_ld, v_ld, o_ld, do_ld, dq_ld, dk_ld, dv_ld;
  const int32_t* key_len;
  int32_t batch, heads, head_dim, tq, tk, causal, dtype;
  float scale;
  int32_t variant;   /* 0 auto (bf16: v3 32x32 swapped MFMA products; f32: v1), 1 v1 (P through LDS),
                        2 v3 with 2-wave workgroups, 3 v3 with 4-wave workgroups (bf16 only) */
  int32_t parts;     /* bwd: 0 dQ and dK / dV, 1 dQ only, 2 dK / dV only (the non-causal bf16 launch,
                        whose two halves share no state: two streams may run them side by side) */
} tt2_attn_args;

/* Alignment diagnostics: probs[b*H + h][q][j] (f32) of a forward already run with these
 * args, recomputed from q, k and the saved lse (exactly 0 where masked). */
int tt2_attn_probs(const tt2_attn_args* a, float* probs, hipStream_t stream);
int tt2_attn_fwd(const tt2_attn_args* a, hipStream_t stream);
int tt2_attn_bwd(const tt2_attn_args* a, hipStream_t stream);

/* ------------------------------------------------------------------ decode
 * One query row per batch element (the AR decode step):
 * out[b*o_ld + 64h ..] = softmax(scale q k^T) v over keys j < n_b of batch b,
 * key j of batch b at k + b*k_bstride + j*k_ld + 64h.  n_b = min(tk, *t_ptr + 1
 * if t_ptr, key_len[b] if key_len): t_ptr is the DEVICE step counter, so the
 * call is replayable from a captured graph. */
typedef struct tt2_attn_decode_args {
  const void* q; const void* k; const void* v; void* out;
  int64_t q_ld, k_bstride, k_ld, v_bstride, v_ld, o_ld;
  const int32_t* key_len;
  const int32_t* t_ptr;
  int32_t batch, heads, head_dim, tk, dtype;
  float scale;
  /* optional early exit: when stop_len != NULL, batch element b is finished once
   * *step >= stop_len[b] (step defaults to t_ptr); its output row is 0 and no key is read */
  const int32_t* stop_len;
  const int32_t* step;
  /* optional fused output projection (wo != NULL): the workgroup of (b, h) also writes
   * slab[(h * batch + b) * heads * head_dim + n] = sum_j o[b, h, j] * wo[n * wo_ld + h * head_dim + j]
   * (f32, n < heads * head_dim): one split-K slab per head for tt2_ln_combine (splits = heads),
   * which adds the bias; out may then be NULL */
  const void* wo;
  int64_t wo_ld;
  float* slab;
  /* optional fused query projection (wq != NULL): q is then the projection INPUT x [batch][q_ld]
   * (heads * head_dim wide) and the head's query is
   * q[b, h, j] = sum_k x[b, k] * wq[(h * head_dim + j) * wq_ld + k] + bq[h * head_dim + j]
   * (f32 accumulation, the query kept in f32): the decoder's cross-attention query GEMM
   * rides in the attention launch */
  const void* wq;
  int64_t wq_ld;
  const float* bq;
  /* optional fused residual combine + LayerNorm of the projection input (ln_part != NULL; needs
   * wq, 8 heads, q_ld == 512, bf16 / f16): the input row is x[b] = LN(q[b] + ln_bias +
   * sum_{s<8} ln_part[(s * batch + b) * 512 + :]) exactly as tt2_ln_combine(splits = 8) computes
   * it (the self-attention's output-projection slabs), and the workgroup of head 0 writes it to
   * ln_out[b] (the next sublayer's residual): the decoder's first post-LN rides in this launch */
  const float* ln_part;
  const float* ln_bias;
  const float* ln_gamma;
  const float* ln_beta;
  void* ln_out;
  float ln_eps;
} tt2_attn_decode_args;
int tt2_attn_decode(const tt2_attn_decode_args* a, hipStream_t stream);
/* cache[b*c_bstride + (*t_ptr)*c_ld + c] = src[b*src_ld + c], c < n */
int tt2_kv_append(const void* src, int64_t src_ld, void* cache, int64_t c_bstride, int64_t c_ld, int n, int batch,
                  const int32_t* t_ptr, int dtype, hipStream_t stream);
/* heads [batch, heads_ld] f32 -> mel_seq[b, t, :], stop_seq[b, t] (+ stop_bias[b, t] if given),
 * prev[b, :] (prev_dtype); stop_len[b] = t + 1 at the first stop logit >= stop_thr (if given);
 * then *t_ptr += 1 and *seed += 1 (seed may be NULL) */
int tt2_decode_emit(const float* heads, int64_t heads_ld, int batch, int n_mels, int t_max, float* mel_seq,
                    float* stop_seq, void* prev, int prev_dtype, int32_t* t_ptr, uint32_t* seed,
                    const float* stop_bias, int32_t* stop_len, float stop_thr, hipStream_t stream);
/* The decode step's whole FFN sublayer in ONE launch (the decoder layer's
 * FFN + third post-LN, modeling_speecht5.py's SpeechT5FeedForward + final_layer_norm):
 *   hidden = relu(x W1^T + b1)            (m x d_ffn, stored in `hidden`, dtype)
 *   slab[s] = hidden[:, 256 s ..] W2[:, 256 s ..]^T   (s < 8, raw f32 partial sums)
 *   y = LN(x + b2 + sum_s slab[s]) * gamma + beta
 * with the arithmetic of the three launches it replaces (tt2_gemm act = relu, tt2_gemm splits = 8
 * main_only, tt2_ln_combine splits = 8): bit-identical results, but slower than those three
 * launches on MI355X (its two in-kernel hand-offs between work groups cost more than two launch
 * boundaries), so the decode step uses it only under schedule 4.  256 work groups that order the
 * three phases among themselves through the counters at `sync` (TT2_FFN_SYNC_INTS int32, zero
 * before the first call; every call leaves them zero again; sync[TT2_FFN_SYNC_ERR] != 0 afterwards
 * means a phase timed out and the outputs are invalid).  m <= 64, d_model 512, d_ffn 2048, dtype TT2_DT_BF16 or TT2_DT_F16,
 * 16-B aligned rows; anything else is TT2_E_INVALID.  Replayable from a captured graph. */
typedef struct tt2_ffn_decode_args {
  const void* x;                      /* [m][512] FFN input and residual */
  const void* w1; const float* b1;    /* [2048][512], [2048] */
  const void* w2; const float* b2;    /* [512][2048], [512] */
  const float* gamma; const float* beta;
  void* hidden;                       /* [m][2048] scratch */
  float* slab;                        /* [8][m][512] scratch */
  int32_t* sync;                      /* [TT2_FFN_SYNC_INTS] */
  void* y;                            /* [m][512] */
  int32_t m, d_model, d_ffn, dtype;
  float eps;
} tt2_ffn_decode_args;
#define TT2_FFN_SYNC_INTS 2048
#define TT2_FFN_SYNC_ERR 1088
int tt2_ffn_decode(const tt2_ffn_decode_args* a, hipStream_t stream);
/* measurement hook: also 8 device wall-clock stamps per work group into stamps[256][8] */
int tt2_ffn_decode_stamps(const tt2_ffn_decode_args* a, uint64_t* stamps, hipStream_t stream);

/* ------------------------------------------------------------ decode step / graph
 * The whole autoregressive decode step (the loop body of
 * modeling_speecht5.py:2215-2267 with a KV cache): pre-net on the previous frame (optional
 * always-on dropout, sites 128 / 129, seed = *seed, bumped every step) -> scaled PE at the
 * device step t -> n_layers x [self-attention with KV-cache append, cross-attention over the
 * encoder memory K/V, FFN, post-LNs] -> mel / stop heads -> frame emit, t += 1.  The library
 * composes the launches itself, so a non-Python host (C++, a JNI / cgo binding) can drive
 * inference; tt2_decode_graph_create captures one step as a hipGraph that the library owns,
 * and tt2_decode_graph_launch replays it n times.
 *
 * Early exit: an utterance finishes at the first frame whose stop logit (+ stop_bias) reaches
 * stop_logit (stop_len[b] = that frame + 1); afterwards its attention reads no keys.  The
 * caller polls stop_len between launches (stop_logit = +inf: forced length).  Frames emitted after
 * an utterance's stop are zero, so a batched post-net sees each utterance zero-padded at its length.
 *
 * Weights are in the step dtype (bf16 / f16 / f32, [out, in] row-major as in the checkpoint);
 * biases, LayerNorm parameters, alpha and the PE table are f32.  All buffers are caller-owned;
 * the workspace (tt2_decode_workspace_size bytes) holds the KV cache and step activations. */
#define TT2_MAX_DEC_LAYERS 16
typedef struct tt2_dec_layer {
  const void* qkv_w; const float* qkv_b;     /* self-attention in_proj [3d, d] */
  const void* o_w; const float* o_b;         /* self-attention out_proj [d, d] */
  const float* ln1_g; const float* ln1_b;
  const void* cq_w; const float* cq_b;       /* cross-attention query rows of in_proj [d, d] */
  const void* co_w; const float* co_b;       /* cross-attention out_proj [d, d] */
  const float* ln2_g; const float* ln2_b;
  const void* ffn1_w; const float* ffn1_b;   /* [F, d] */
  const void* ffn2_w; const float* ffn2_b;   /* [d, F] */
  const float* ln3_g; const float* ln3_b;
} tt2_dec_layer;

typedef struct tt2_decode_desc {
  int32_t batch, text_len, t_max, n_layers, d_model, n_heads, d_ffn, n_mels, prenet_dim;
  int32_t dtype;        /* step storage type: TT2_DT_BF16, TT2_DT_F16 (batch <= 64) or TT2_DT_F32 */
  int32_t schedule;     /* 0 auto, 1 plain (one launch per op), 2 split-K (16-bit, batch <= 64; output
                         * projections fused into the attention launches), 3 split-K without that
                         * fusion, 4 split-K with it and each FFN sublayer as one tt2_ffn_decode
                         * launch (bit-identical to 2, measured slower: opt-in) */
  float ln_eps;
  float prenet_dropout; /* 0 = off (Tacotron2 keeps it on at inference) */
  float stop_logit;     /* logit(stop_threshold); +inf never stops */
  const void* fc1_w; const float* fc1_b;     /* pre-net [P, n_mels], [P, P], proj [d, P] */
  const void* fc2_w; const float* fc2_b;
  const void* proj_w; const float* proj_b;
  const float* alpha;                        /* decoder PE scale (device scalar) */
  const float* pe_table;                     /* [>= t_max + 1][d] */
  tt2_dec_layer layers[TT2_MAX_DEC_LAYERS];
  const void* heads_w; const float* heads_b; /* [n_mels + 1, d]: mel rows, then the stop row */
  const void* mem_kv;        /* [batch * text_len, n_layers * 2d]: layer l's K at column 2dl, V at 2dl + d */
  const int32_t* text_lens;  /* [batch] phonemes per utterance */
  float* mel_seq;            /* out [batch][t_max][n_mels] (pre-post-net frames) */
  float* stop_seq;           /* out [batch][t_max] */
  int32_t* stop_len;         /* out [batch]; INT32_MAX while running */
  const float* stop_bias;    /* optional [batch][t_max] */
  int32_t* step;             /* device step counter */
  uint32_t* seed;            /* device dropout seed */
  void* workspace; size_t ws_bytes;
} tt2_decode_desc;
typedef struct tt2_decode_graph* tt2_decode_graph_t;

size_t tt2_decode_workspace_size(const tt2_decode_desc* d);
/* step = 0, seed = seed0, previous frame = 0 (the go frame), stop_len = INT32_MAX */
int tt2_decode_reset(const tt2_decode_desc* d, uint32_t seed0, hipStream_t stream);
/* one step as eager launches */
int tt2_decode_step(const tt2_decode_desc* d, hipStream_t stream);
int tt2_decode_graph_create(const tt2_decode_desc* d, hipStream_t stream, tt2_decode_graph_t* out);
/* also captures `steps` (1..64) consecutive steps as a second graph: a launch of n steps then
 * replays it n / steps times (one graph boundary per `steps` frames) and the one-step graph for
 * the rest.  tt2_decode_graph_create == steps 1. */
int tt2_decode_graph_create_n(const tt2_decode_desc* d, int32_t steps, hipStream_t stream, tt2_decode_graph_t* out);
/* n_steps replays.  The device step counter saturates at t_max: replays past it write no
 * KV-cache row, emit no frame and leave every output unchanged. */
int tt2_decode_graph_launch(tt2_decode_graph_t g, int32_t n_steps, hipStream_t stream);
int tt2_decode_graph_destroy(tt2_decode_graph_t g);

/* ------------------------------------------------------------- reductions */
#define TT2_COLSUM_ROWS 128
#define TT2_BN_ROWS_PER_CHUNK 64
#define TT2_PE_BWD_BLOCKS 1024
#define TT2_LOSS_BLOCKS 1024
#define TT2_ADAM_NORM_BLOCKS 1024

/* dst[c] = beta*dst[c] + sum_r src[r*ld + c] (fixed summation order) */
typedef struct tt2_reduce_args {
  const float* src; float* dst;
  int64_t ld; int32_t rows, cols;
  float beta;
} tt2_reduce_args;
int tt2_reduce_rows(const tt2_reduce_args* a, hipStream_t stream);

/* Bias gradient: dst[n] = beta*dst[n] + sum_m x[m*ld + n]. */
size_t tt2_colsum_workspace_size(int m, int n);
int tt2_colsum(const void* x, int dtype, int64_t ld, int m, int n, float* dst, float beta, void* ws,
               size_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------------------- LayerNorm
 * fwd: y = LN(x + drop(branch)) (branch may be NULL), mean/rstd [m] f32 saved.
 * bwd: dx = dL/ds (residual stream), dbranch = drop'(dx); dgamma/dbeta (f32)
 *      = grad_beta*old + sum over rows.  C must be 512 (d_model).
 * Replaces the post-LN residual blocks of SURVEY 8(a) a3, a4, a6, a7. */
typedef struct tt2_ln_args {
  const void* x; const void* branch; const void* dy;
  void* y; void* dx; void* dbranch;
  const float* gamma; const float* beta;
  float* mean; float* rstd;
  float* dgamma; float* dbeta;
  void* workspace; size_t ws_bytes;
  const uint32_t* drop_seed;
  int32_t m, c, dtype;
  float eps, grad_beta;
  uint32_t drop_site, drop_thr;
  float drop_scale;
  float* dbias;   /* bwd, optional: grad_beta*dbias + column sums of the branch gradient
                     (= the bias gradient of the linear layer that produced `branch`) */
  int32_t defer_finalize;   /* bwd: leave the per-workgroup column partials in `workspace`
                               and do not write dgamma/dbeta/dbias yet: a later
                               tt2_layernorm_bwd (finalize_prev) or
                               tt2_layernorm_bwd_finalize completes them */
  const struct tt2_ln_args* finalize_prev;   /* bwd, optional: a deferred earlier call
                               (same c) whose dgamma/dbeta/dbias this launch completes in its
                               spare lanes; its workspace must not have been reused since */
} tt2_ln_args;
int tt2_layernorm_fwd(const tt2_ln_args* a, hipStream_t stream);
size_t tt2_layernorm_bwd_workspace_size(const tt2_ln_args* a);
/* tt2_gemm_grouped that also completes `fin`, a deferred LayerNorm backward (defer_finalize
 * = 1, partials still in its workspace), inside the group's split-K reduce launch: a layer's
 * last LayerNorm gradients need no launch of their own.  fin may be NULL; n may be 0. */
int tt2_gemm_grouped_fin(const tt2_gemm_args* probs, int32_t n, const tt2_ln_args* fin, hipStream_t stream);
/* tt2_gemm_grouped_fin with at most max_groups work groups at a time (rounded down to a multiple
 * of 8; 0: every 256 x 128 item at once): the items go out as consecutive launches of that many,
 * so a launch beside other work on a second stream leaves the remaining CUs to that work. */
int tt2_gemm_grouped_ex(const tt2_gemm_args* probs, int32_t n, const tt2_ln_args* fin, int32_t max_groups,
                        hipStream_t stream);
int tt2_layernorm_bwd(const tt2_ln_args* a, hipStream_t stream);
/* Completes a deferred tt2_layernorm_bwd (defer_finalize = 1): dgamma/dbeta/dbias from the
 * partials it left in a->workspace.  Same fixed summation order as a chained finalize. */
int tt2_layernorm_bwd_finalize(const tt2_ln_args* a, hipStream_t stream);
/* Decode-step residual combine + LayerNorm (x / y of dtype bf16 or f16, c = 512):
 *   y[m, :] = LN(x[m, :] + bias + sum_{s < splits} part[s][m][:]) * gamma + beta
 * part: the raw f32 partial slabs [splits][m][c] of a skinny split-K projection (tt2_gemm
 * with splits > 1 and main_only; splits 1, 2, 4, 8 or 16), summed in a fixed order.
 * Replaces the output-projection epilogue + residual + LayerNorm of a decoder sublayer
 *  where splitting K spreads the weight stream over more CUs. */
int tt2_ln_combine(const void* x, const float* part, int32_t splits, const float* bias, const float* gamma,
                   const float* beta, void* y, int32_t m, int32_t c, float eps, int32_t dtype, hipStream_t stream);

/* ------------------------------------------------------------- BatchNorm
 * fwd: out = drop(act((y - mean)*rstd*gamma + beta)) (+ res), statistics over
 *      all m rows (training: batch stats + running update; eval: running stats).
 * bwd: dy from dout (dtype dout_dtype), dgamma/dbeta written (f32).
 * Replaces the Conv1d+BatchNorm blocks of SURVEY 8(a) a1 (relu) and a9 (tanh). */
typedef struct tt2_bn_args {
  const void* y; const void* dout; const void* res;
  void* out; void* dy;
  const float* gamma; const float* beta;
  float* mean; float* rstd;
  float* run_mean; float* run_var;
  float* dgamma; float* dbeta;
  void* workspace; size_t ws_bytes;
  const uint32_t* drop_seed;
  int64_t res_ld;  /* row stride of res (elements) */
  int32_t m, c, act, dtype, out_dtype, res_dtype, dout_dtype, training;
  float eps, momentum;
  uint32_t drop_site, drop_thr;
  float drop_scale;
  /* SyncBatchNorm (the *_stats / *_apply phases below; ignored by tt2_batchnorm_fwd/bwd) */
  float* sync_buf;               /* tt2_batchnorm_sync_size bytes, 16-B aligned */
  int32_t sync_world, sync_rank;
  /* stats_rows > 0 says the workspace already holds this pass's per-chunk column statistics in
   * chunks of stats_rows rows, so the statistics pass over the rows is skipped: the training
   * forward's moments of y (tt2_gemm col_stats) or the backward's sums (tt2_gemm bn_bwd; both
   * with stats_rows = TT2_GEMM_STATS_ROWS); tt2_batchnorm_workspace_size then gives that layout's
   * size.  0: the pass runs (its own chunking). */
  int32_t stats_rows;
} tt2_bn_args;
size_t tt2_batchnorm_workspace_size(const tt2_bn_args* a);
int tt2_batchnorm_fwd(const tt2_bn_args* a, hipStream_t stream);
int tt2_batchnorm_bwd(const tt2_bn_args* a, hipStream_t stream);
/* SyncBatchNorm over sync_world data-parallel ranks, rank r holding its own m_r rows (ranks
 * may differ: torch.nn.SyncBatchNorm's semantics, training statistics and the backward's
 * column sums over all sum_r m_r rows, each rank weighted by its row count; the dgamma / dbeta
 * parameter gradients stay this rank's sums, for the gradient all-reduce).
 * Each pass is two phases around a caller-issued SUM all-reduce of the first
 * sync_world * 3 * c floats of sync_buf ([W][3][c]: this rank's slot holds its moments / sums
 * and its row count m, the other slots zeros, so the reduced slots are exact and rank-ordered
 * on every rank):
 *   tt2_batchnorm_fwd_stats -> all-reduce -> tt2_batchnorm_fwd_apply   (training only)
 *   tt2_batchnorm_bwd_stats -> all-reduce -> tt2_batchnorm_bwd_apply
 * sync_world = 1 reproduces tt2_batchnorm_fwd / _bwd (no exchange needed).  The optional
 * SyncBN of SURVEY.md:219 (per-replica statistics stay the default). */
size_t tt2_batchnorm_sync_size(const tt2_bn_args* a);
int tt2_batchnorm_fwd_stats(const tt2_bn_args* a, hipStream_t stream);
int tt2_batchnorm_fwd_apply(const tt2_bn_args* a, hipStream_t stream);
int tt2_batchnorm_bwd_stats(const tt2_bn_args* a, hipStream_t stream);
int tt2_batchnorm_bwd_apply(const tt2_bn_args* a, hipStream_t stream);

/* -------------------------------------------------- embedding / pos. enc. */
int tt2_embedding_fwd(const int64_t* ids, const void* table, void* out, int m, int c, int vocab, int dtype,
                      hipStream_t stream);
/* dtable (f32) row v = sum of dout rows with ids == v, added in increasing row order (gathered per
 * table row: deterministic, no atomics); every row is written; rows == pad_idx get zero */
int tt2_embedding_bwd(const int64_t* ids, const void* dout, float* dtable, int m, int c, int vocab, int pad_idx,
                      int dtype, hipStream_t stream);

/* out = drop(x + alpha*pe[row % t + t_offset (+ *t_ptr if t_ptr)]); bwd: dx = drop'(dout),
 * *dalpha = sum dx*pe */
typedef struct tt2_pe_args {
  const void* x; const void* dout; void* out; void* dx;
  const float* alpha; const float* pe; float* dalpha;
  void* workspace; size_t ws_bytes;
  const uint32_t* drop_seed;
  const int32_t* t_ptr;
  int32_t m, c, t, t_offset, dtype;
  uint32_t drop_site, drop_thr;
  float drop_scale;
} tt2_pe_args;
int tt2_posenc_fwd(const tt2_pe_args* a, hipStream_t stream);
size_t tt2_posenc_bwd_workspace_size(void);
int tt2_posenc_bwd(const tt2_pe_args* a, hipStream_t stream);

/* teacher forcing: out[b*t + j] = j == 0 ? 0 : mel[b, j-1] (mel f32 [batch, t, c]) */
int tt2_shift_right(const float* mel, void* out, int batch, int t, int c, int dtype, hipStream_t stream);
int tt2_cast2d(const void* src, int src_dtype, int64_t src_ld, void* dst, int dst_dtype, int64_t dst_ld, int m,
               int n, hipStream_t stream);

/* ------------------------------------------------------------------- loss
 * heads [batch*t, heads_ld] f32 (cols 0..n_mels-1 mel_before, col n_mels stop logit),
 * mel_after [batch*t, n_mels] f32, target f32 [batch, t, n_mels].
 * loss_out[4] = (total, mse_before, mse_after, bce_stop); gradients: g_heads
 * (f32, heads_ld; mel cols carry before + after terms), g_after (grad_dtype).
 * Replaces SURVEY 8(a) a10. */
typedef struct tt2_loss_args {
  const float* heads; const float* mel_after; const float* target;
  const int32_t* mel_len;
  float* loss_out; float* g_heads; void* g_after;
  void* workspace; size_t ws_bytes;
  int64_t heads_ld;
  int32_t batch, t, n_mels, grad_dtype;
  float pos_weight;
  float grad_scale;  /* multiplies every gradient (1/world_size under data parallelism) */
  int32_t separate_grads;  /* 1: g_heads' mel columns hold only d/d(mel_before) (no residual
                              d/d(mel_after) term folded in): the autograd boundary's layout */
} tt2_loss_args;
size_t tt2_loss_workspace_size(void);
int tt2_tts_loss(const tt2_loss_args* a, hipStream_t stream);

/* conv dgrad weight: wd[ci][tap][co] = w[co][k-1-tap][ci] */
int tt2_conv_weight_flip(const void* w, void* wd, int cout, int cin, int k, int dtype, hipStream_t stream);
/* The same flip for up to TT2_WFLIP_MAX conv layers in one launch (the backward flips every
 * encoder / post-net conv weight once per step). */
#define TT2_WFLIP_MAX 16
typedef struct tt2_wflip_job {
  const void* w; void* wd;
  int32_t cout, cin, k, pad_;
} tt2_wflip_job;
int tt2_conv_weight_flip_batch(const tt2_wflip_job* jobs, int32_t n, int32_t dtype, hipStream_t stream);

/* -------------------------------------------------------------- optimizer
 * Fused Adam(W) over the flat f32 parameter buffer with optional global-norm
 * clipping and Noam warmup (lr * d^-0.5 * min(s^-0.5, s*warmup^-1.5)); writes the
 * bf16 shadow used by the bf16 kernels.  step is a device counter (step+1 is used). */
typedef struct tt2_adam_args {
  float* params; const float* grads; float* exp_avg; float* exp_avg_sq;
  void* shadow_bf16;
  int32_t* step;
  void* workspace; size_t ws_bytes;
  int64_t n;
  float lr, beta1, beta2, eps, weight_decay, clip_norm, warmup;
  int32_t noam, d_model;
  /* clip: norm_parts != NULL gives the squared gradient norm as the sum of norm_nparts partial
   * sums the caller computed beforehand (tt2_sumsq_parts over ranges that cover grads[0, n)),
   * in place of the step's own pass over the gradients */
  const float* norm_parts;
  int32_t norm_nparts;
  /* gate != NULL: the update runs only while *gate != 0 (the pipelined optimizer's deferred
   * Adam: armed by tt2_adam_gate(op 1) when a step's gradients are final, consumed by
   * tt2_adam_gate(op 0) once the deferred update has run), so a captured step replays a
   * deferred update exactly once however often it was flushed eagerly in between */
  const int32_t* gate;
} tt2_adam_args;
size_t tt2_adam_workspace_size(void);
int tt2_adam_step(const tt2_adam_args* a, hipStream_t stream);
/* parts[0 .. nparts) = partial sums of g[i]^2 over g[0, n) (fixed split: reproducible) */
int tt2_sumsq_parts(const float* g, int64_t n, float* parts, int32_t nparts, hipStream_t stream);
/* step += 1; seed += 1 (either may be NULL: the pipelined optimizer bumps the dropout seed at the
 * end of a step and the step counter once the deferred Adam has run) */
int tt2_step_bump(int32_t* step, uint32_t* seed, hipStream_t stream);
/* op 1 (arm): *gate = 1.  op 0 (consume): if *gate != 0 { *step += 1 (when step != NULL); *gate = 0 } */
int tt2_adam_gate(int32_t* gate, int32_t* step, int32_t op, hipStream_t stream);

/* ---------------------------------------------------------- capture hygiene
 * For each of n streams, status[i] = 0: not part of the origin's capture, 1: part of it and
 * joined (the origin depends on all its captured work), 2: part of it with captured work the
 * origin does not depend on (ending the capture now would leave it unjoined), 3: its capture
 * was invalidated.  The origin stream must be capturing.  Host-only (reads the graph being
 * captured; enqueues nothing). */
int tt2_capture_joined(hipStream_t origin, const hipStream_t* streams, int32_t n, int32_t* status);

/* ---------------------------------------------------------- block-level entry points
 * One call per block of the path: each is a fixed sequence of the kernels
 * above on the caller's stream, with the block's shape and options in a tt2_desc.
 * Layout: activations channels-last [rows = batch * tq (or tk), channels] of desc.dtype
 * (TT2_DT_BF16 or TT2_DT_F32); weights of desc.dtype in nn.Linear layout [out][in]
 * (conv: [c_out][kernel][c_in], see tt2_conv_weight_pack); biases, LayerNorm / BatchNorm
 * parameters, statistics and every weight / bias gradient f32.  Weight and bias
 * gradients are written (not accumulated).
 *  - `saved`: activations a forward keeps for its backward, tt2_<block>_saved_size() bytes,
 *    written by _fwd and read by _bwd (the caller keeps it between them);
 *  - `workspace`: scratch of tt2_<block>_workspace_size() bytes (split-K slabs, partials),
 *    free again when the call's work has finished on the stream.
 * Dropout: p = desc.dropout at hash site desc.site (the FFN's second site is site + 1)
 * with seed *desc.seed, applied when desc.training is set. */
typedef struct tt2_desc {
  int32_t batch;          /* B */
  int32_t tq;             /* rows per utterance: query / sequence length */
  int32_t tk;             /* attention keys per utterance (cross: memory length; self: = tq) */
  int32_t d_model;        /* 512 (heads of width 64) */
  int32_t n_heads;
  int32_t d_ffn;
  int32_t c_in, c_out;    /* linear / conv1d_bn_act / heads channels (heads: c_out = n_mels + 1) */
  int32_t kernel;         /* conv taps (odd; "same" padding (kernel - 1) / 2) */
  int32_t dtype;          /* TT2_DT_BF16 or TT2_DT_F32 */
  int32_t causal;         /* attention: causal mask (self-attention) */
  int32_t cross;          /* attention: 1 = Q from x, K / V from mem (in_proj rows 0:d / d:3d) */
  int32_t act;            /* conv1d_bn_act: 0 none, 1 relu, 2 tanh */
  int32_t training;       /* dropout on; BatchNorm batch statistics + running-stat update */
  float eps;              /* LayerNorm / BatchNorm epsilon */
  float momentum;         /* BatchNorm running-stat momentum */
  float dropout;          /* p (0 = none) */
  const uint32_t* seed;   /* device dropout seed */
  uint32_t site;          /* dropout hash site */
  const int32_t* k_len;   /* [batch] valid keys per utterance (key padding mask) or NULL */
  const int32_t* mel_len; /* loss: [batch] valid frames */
  int32_t n_mels;         /* loss / heads: mel channels (80) */
  int32_t heads_ld;       /* heads / loss: row stride of the heads buffer (>= n_mels + 1) */
  float pos_weight;       /* loss: BCE positive weight */
  float grad_scale;       /* loss: multiplies every gradient (1 / world under data parallelism) */
} tt2_desc;

/* Attention sublayer (SURVEY 8(a) a3 / a6 / a7 + residual + post-LN):
 *   y = LN(x + drop(out_proj(SDPA(q = x Wq^T + bq, k|v = src Wkv^T + bkv))) ; src = cross ? mem : x
 * w_in [3d][d] (nn.MultiheadAttention in_proj), b_in [3d], w_out [d][d], b_out [d], ln_g / ln_b [d].
 * bwd: dy -> dx (residual + query path; + key/value path when not cross), dmem (cross: the
 * key/value path; NULL otherwise), and the parameter gradients. */
size_t tt2_attn_block_saved_size(const tt2_desc* d);
size_t tt2_attn_block_workspace_size(const tt2_desc* d);
int tt2_attn_block_fwd(const tt2_desc* d, const void* x, const void* mem, const void* w_in, const float* b_in,
                       const void* w_out, const float* b_out, const float* ln_g, const float* ln_b, void* y,
                       void* saved, void* workspace, size_t ws_bytes, hipStream_t stream);
int tt2_attn_block_bwd(const tt2_desc* d, const void* x, const void* mem, const void* w_in, const void* w_out,
                       const float* ln_g, const float* ln_b, const void* saved, const void* dy, void* dx, void* dmem,
                       float* dw_in, float* db_in, float* dw_out, float* db_out, float* dln_g, float* dln_b,
                       void* workspace, size_t ws_bytes, hipStream_t stream);

/* Position-wise FFN sublayer:
 *   y = LN(x + drop_{site+1}(drop_{site}(relu(x W1^T + b1)) W2^T + b2)),  w1 [d_ffn][d], w2 [d][d_ffn]. */
size_t tt2_ffn_saved_size(const tt2_desc* d);
size_t tt2_ffn_workspace_size(const tt2_desc* d);
int tt2_ffn_fwd(const tt2_desc* d, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                const float* ln_g, const float* ln_b, void* y, void* saved, void* workspace, size_t ws_bytes,
                hipStream_t stream);
int tt2_ffn_bwd(const tt2_desc* d, const void* x, const void* w1, const void* w2, const float* ln_g,
                const float* ln_b, const void* saved, const void* dy, void* dx, float* dw1, float* db1, float* dw2,
                float* db2, float* dln_g, float* dln_b, void* workspace, size_t ws_bytes, hipStream_t stream);

/* Linear (pre-net / projections): y [rows][c_out] = x [rows][c_in] W^T + b (b may be NULL). */
size_t tt2_linear_workspace_size(const tt2_desc* d);
int tt2_linear_fwd(const tt2_desc* d, const void* x, const void* w, const float* b, void* y, void* workspace,
                   size_t ws_bytes, hipStream_t stream);
int tt2_linear_bwd(const tt2_desc* d, const void* x, const void* w, const void* dy, void* dx, float* dw, float* db,
                   void* workspace, size_t ws_bytes, hipStream_t stream);

/* Residual add + post-LayerNorm: y = LN(x + drop(branch)) over d_model channels; saved = mean / rstd.
 * bwd: dx = dL/d(x + drop(branch)), dbranch = drop'(dx), dln_g / dln_b. */
size_t tt2_add_ln_saved_size(const tt2_desc* d);
size_t tt2_add_ln_workspace_size(const tt2_desc* d);
int tt2_add_ln_fwd(const tt2_desc* d, const void* x, const void* branch, const float* ln_g, const float* ln_b,
                   void* y, void* saved, hipStream_t stream);
int tt2_add_ln_bwd(const tt2_desc* d, const void* x, const void* branch, const float* ln_g, const void* saved,
                   const void* dy, void* dx, void* dbranch, float* dln_g, float* dln_b, void* workspace,
                   size_t ws_bytes, hipStream_t stream);

/* Conv1d + BatchNorm + activation + dropout (SURVEY 8(a) a1 encoder pre-net, a9 post-net):
 *   out = drop(act(BN(conv(x) + b))) (+ res, [rows][c_out] of res_dtype, when res != NULL);
 * w [c_out][kernel][c_in]; BN over all rows (training: batch statistics, run_mean / run_var
 * updated; eval: the running statistics).  bwd: dout -> dx and dw / db / dbn_g / dbn_b. */
size_t tt2_conv1d_bn_act_saved_size(const tt2_desc* d);
size_t tt2_conv1d_bn_act_workspace_size(const tt2_desc* d);
int tt2_conv1d_bn_act_fwd(const tt2_desc* d, const void* x, const void* w, const float* b, const float* bn_g,
                          const float* bn_b, float* run_mean, float* run_var, const void* res, int32_t res_dtype,
                          void* out, void* saved, void* workspace, size_t ws_bytes, hipStream_t stream);
int tt2_conv1d_bn_act_bwd(const tt2_desc* d, const void* x, const void* w, const float* bn_g, const float* bn_b,
                          const void* saved, const void* dout, void* dx, float* dw, float* db, float* dbn_g,
                          float* dbn_b, void* workspace, size_t ws_bytes, hipStream_t stream);
/* nn.Conv1d weight [c_out][c_in][k] -> the blocks' tap-major [c_out][k][c_in] (same dtype) */
int tt2_conv_weight_pack(const void* w, void* wp, int32_t cout, int32_t cin, int32_t k, int32_t dtype,
                         hipStream_t stream);

/* Mel + stop heads: heads [rows][heads_ld] f32, cols 0..n_mels-1 = mel_before,
 * col n_mels = stop logit; w [n_mels + 1][d_model] (mel_linear rows, then stop_linear), b f32.
 * bwd: g_heads (f32, same layout) -> dx, dw, db. */
size_t tt2_heads_workspace_size(const tt2_desc* d);
int tt2_heads_fwd(const tt2_desc* d, const void* x, const void* w, const float* b, float* heads, void* workspace,
                  size_t ws_bytes, hipStream_t stream);
int tt2_heads_bwd(const tt2_desc* d, const void* x, const void* w, const float* g_heads, void* dx, float* dw,
                  float* db, void* workspace, size_t ws_bytes, hipStream_t stream);

/* Loss over rows = batch * tq: loss_out[4] = (total, mse_before, mse_after, bce);
 * bwd also writes g_heads (d/d mel_before in cols < n_mels, d/d stop logit in col n_mels) and
 * g_after (d/d mel_after, desc.dtype). */
size_t tt2_loss_block_workspace_size(const tt2_desc* d);
int tt2_loss_fwd(const tt2_desc* d, const float* heads, const float* mel_after, const float* target,
                 float* loss_out, void* workspace, size_t ws_bytes, hipStream_t stream);
int tt2_loss_bwd(const tt2_desc* d, const float* heads, const float* mel_after, const float* target,
                 float* loss_out, float* g_heads, void* g_after, void* workspace, size_t ws_bytes,
                 hipStream_t stream);

/* Data-parallel gradient bucket: in-place SUM all-reduce of n elements of
 * dtype over an RCCL communicator (ncclComm_t) on the caller's stream.  librccl is bound at
 * the first call (dlopen); the communicator helpers below wrap ncclGetUniqueId /
 * ncclCommInitRank / ncclCommDestroy for hosts without torch.distributed. */
int tt2_allreduce_bucket(void* buf, size_t n, int32_t dtype, void* comm, hipStream_t stream);
int tt2_comm_unique_id(void* id_out /* 128 bytes */);
int tt2_comm_init(void** comm_out, int32_t nranks, const void* id /* 128 bytes */, int32_t rank);
int tt2_comm_destroy(void* comm);
/* Measurement stand-in for one bucket's exchange at N ranks (tt2/dist.py StandinGradSync; the
 * DP schedule rehearsed on one GPU): `wgs` work groups copy `bytes` from src to scratch, then each
 * holds its CU until `seconds` have passed since it started.  No communicator; src is not modified.
 * rec (optional, 2 * wgs u64): each work group's {start, end} on the device wall clock. */
int tt2_comm_standin(const void* src, void* scratch, size_t bytes, double seconds, int32_t wgs, uint64_t* rec,
                     hipStream_t stream);

/* ------------------------------------------------------------ audio data path
 * Either side of the mel engine: log-mel extraction of the
 * training targets and Griffin-Lim inversion of synthesised mels.  The STFT, inverse DFT
 * and mel projections are tt2_gemm calls (f32) on window-folded bases; these are the
 * byte-moving steps around them (all f32, caller-owned buffers, caller's stream).
 * Frame layout: utterance b's padded signal is padded[b * Lp ...] with Lp a multiple of
 * hop, so the batch's frames are one strided matrix (row r at sample r * hop, ld = hop) and
 * utterance b owns rows [b * R, b * R + n_frames_b), R = Lp / hop.  Replaces the reference
 * pipeline's librosa / torch.stft feature extraction and its vocoder hand-off. */
/* padded[b][j] = x[b][reflect(j - pad)] for j < len_b + 2 pad (np.pad "reflect"), else 0;
 * lens may be NULL (all len); pad < len. */
int tt2_reflect_pad(const float* x, int64_t ldx, const int32_t* lens, int32_t batch, int32_t len, float* padded,
                    int64_t padded_len, int32_t pad, hipStream_t stream);
/* mag[r][k] = |spec[r][k] + i spec[r][n_bins + k]| (k < n_bins), zero padding to ld_mag. */
int tt2_spec_magnitude(const float* spec, int64_t ld_spec, int32_t m, int32_t n_bins, float* mag, int64_t ld_mag,
                       hipStream_t stream);
/* out = mag * e / |e| as [re | im] rows (phase 0 where est is NULL or e == 0): Griffin-Lim's
 * projection onto the target magnitude. */
int tt2_spec_rephase(const float* mag, int64_t ld_mag, const float* est, int64_t ld_est, int32_t m, int32_t n_bins,
                     float* out, int64_t ld_out, hipStream_t stream);
/* y[b][t] = sum_f frames[b * R + f][t + n_fft/2 - f hop] / sum_f hann^2(...) for t < len_b
 * (least-squares iSTFT overlap-add, centre padding removed), 0 beyond. */
int tt2_overlap_add(const float* frames, int64_t ld_frames, const int32_t* lens, int32_t batch, int32_t len,
                    int32_t rows_per_utt, int32_t n_fft, int32_t hop, float* y, int64_t ld_y, hipStream_t stream);
/* scatter = 0: mel[b][t][c] = log(max(rows[b * R + t][c], clamp)) (t < frames_b, else log clamp);
 * scatter = 1: rows[b * R + t][c] = exp(mel[b][t][c]) (t < frames_b, else 0).  mel [batch][t][n_mels]. */
int tt2_mel_rows(float* rows, int64_t ld_rows, float* mel, const int32_t* frames, int32_t batch, int32_t t,
                 int32_t n_mels, int32_t rows_per_utt, float clamp, int32_t scatter, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
