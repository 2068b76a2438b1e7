/*
 * zonos_hip.h — C ABI of libzonos_hip.so, the MI355X (gfx950) hot path of Zonos generate() +
 * DACAutoencoder.decode().
 *
 * The reference (BreakTheBeta/Zonos_Vibes) is pure Python with no FFI; its device work is
 * ATen ops called from the functions cited below. This ABI is the boundary the Python host
 * (zonos_vibes_amd/) binds with ctypes to replace them. Conventions:
 *   - every pointer is a device pointer owned by the caller (allocated by torch), unless noted;
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream);
 *   - every function returns 0 on success or a nonzero status; zmi_last_error() explains it;
 *   - no function allocates or synchronises, so every launcher can be hipGraph-captured;
 *   - gfx950 only: several launchers size their workgroups for its 160 KB of LDS (the SSD prefill scan ~148 KB, the
 *     staged split-K GEMM ~132 KB, the DAC's staged convs up to 156 KB) and return an error, with no smaller-LDS
 *     fallback, where the device grants less.
 */
#ifndef ZONOS_HIP_H
#define ZONOS_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------------
 * Weight-streaming GEMV / skinny GEMM:  out[m, n] = sum_k A[m, k] W[n, k]  (+ fused epilogue)
 * Replaces nn.Linear in zonos/backbone/_torch.py:114-115 (in_proj/out_proj), :147-152 (fc1/fc2)
 * and zonos/model.py:100-101 (apply_heads); the LayerNorm prologue replaces nn.LayerNorm at
 * _torch.py:62,88,90 (norm, norm2, norm_f).
 * ------------------------------------------------------------------------------------- */
enum {
  ZMI_EPI_STORE = 0,    /* out bf16 [M][ldo]                                                   */
  ZMI_EPI_RESIDUAL = 1, /* out bf16 [M][ldo] += bf16(acc)          (_torch.py:100-101)          */
  ZMI_EPI_QKV = 2,      /* q -> out, rope(k) / v -> KV cache        (_torch.py:18-49, 117-126)  */
  ZMI_EPI_SWIGLU = 3,   /* out bf16 [M][F] = y * silu(gate)        (_torch.py:150-152)          */
  ZMI_EPI_LOGITS = 4,   /* out f32 [M][9][1026] = bf16(acc).float() (model.py:100-101,111)      */
  ZMI_EPI_F32 = 5       /* out f32 [M][ldo] raw fp32 sums (tests)                              */
};
enum { ZMI_PACK_IDENTITY = 0, ZMI_PACK_SWIGLU = 1 };
/* prologue of the activation rows (ZmiGemvArgs.pro):
 *   AUTO   LayerNorm if ln_w, else the rows as they are;
 *   ADDLN  mamba-ssm layer_norm_fn(X, ln_w, ln_b, residual = aux, prenorm=True): s = X + aux in fp32,
 *          LayerNorm(s); res_out (may be NULL) <- bf16(s), written by one workgroup per row tile
 *          (res_out must not alias aux: other workgroups still read aux);
 *   GRMS   mamba-ssm RMSNormGated(X, z) * ln_w (norm_before_gate=False, one group), aux = the f32 gate
 *          z * sigmoid(z) (zmi_mamba2_step's gz), at most 4 rows. */
enum { ZMI_PRO_AUTO = 0, ZMI_PRO_ADDLN = 2, ZMI_PRO_GRMS = 3, ZMI_PRO_GRMS_G = 4 };

typedef struct ZmiGemvArgs {
  const void* W;        /* packed weight (zmi_pack_weight, layout M8)                          */
  const void* X;        /* bf16 [M][ldx] activations                                          */
  int M, N, K, ldx;     /* N = packed (padded) columns, multiple of 8; K in {512 .. 8192}, pow2  */
  int groups;           /* 8-column groups per workgroup: 0 = library choice, else 1 or 2      */
  int reserved;
  const void* ln_w;     /* bf16 [K] LayerNorm weight, or NULL for a plain GEMV                */
  const void* ln_b;     /* bf16 [K] LayerNorm bias                                             */
  float eps;
  void* out;
  int ldo;
  int n_valid;          /* real (unpadded) columns                                             */
  const int* row_kv;    /* QKV: [M] KV-cache row of each activation row                        */
  const int* row_pos;   /* QKV: [M] position (<0: inactive row, nothing written)               */
  void* k_cache;        /* QKV: bf16 K cache [rows][hkv][smax][hd] of this layer               */
  void* v_cache;        /* QKV: bf16 V cache, transposed: [rows][hkv][hd][smax]                 */
  int smax, hq, hkv, hd;
  const float* rope;    /* [16384][hd/2][2] (cos, sin) fp32 (_torch.py:9-15)                  */
  void* diag;           /* NULL; diagnostic builds only (-DZMI_GEMV_STAMPS): phase stamps       */
  int pro;              /* ZMI_PRO_*                                                            */
  int ld_aux;           /* row stride of aux and res_out (elements)                             */
  const void* aux;      /* ADDLN: bf16 residual rows; GRMS: f32 gate rows z * sigmoid(z); GRMS_G: f32 rows g = y * gate (X unused) */
  void* res_out;        /* ADDLN: bf16 [M][ld_aux] new residual, or NULL                         */
} ZmiGemvArgs;

int zmi_pack_weight(const void* src, void* dst, int n_src, int k, int n_pad, int mode, void* stream);
/* One kernel for every M: a row's result is bit-identical whatever the batch it is computed in. */
int zmi_gemv_launch(const ZmiGemvArgs* args, int epi, void* stream);
/* Many-row fc2 (K = 8192) or out_proj (K = 2048), EPI_RESIDUAL, plain (reference _torch.py:100-101,141,152), or
 * the hybrid's Mamba2 out_proj (K = 4096 = d_ssm, EPI_STORE: mamba_ssm out_proj of the prefill): a split-K GEMM
 * (one workgroup per 64-column block, K segment -- 8 x 1024 / 4 x 1024 / 4 x 512, the GEMV's wave split -- and
 * row group, ZMI_OPT_SPLITK_WGS), fp32 segment sums in `part`, then a reduce launch adding the segments in K
 * order + the residual / store epilogue. Bit-identical to zmi_gemv_launch for every row (the GEMV's per-segment
 * MFMA chains and segment order); reads the activation rows once per column block instead of once per column
 * group. part: zmi_gemv_splitk_floats(M, N) floats. */
int zmi_gemv_splitk(const ZmiGemvArgs* args, int epi, float* part, int64_t part_floats, void* stream);
/* The same with ln_w != NULL (N = 2048): the reduce also writes LayerNorm(new row; ln_w, ln_b, eps) to xn [M][ldxn],
 * bit-identical to zmi_layernorm_rows of the new rows, so the next op's LayerNorm pre-pass is not launched. */
int zmi_gemv_splitk_ln(const ZmiGemvArgs* args, int epi, float* part, int64_t part_floats, const void* ln_w,
                       const void* ln_b, float eps, void* xn, int ldxn, void* stream);
int64_t zmi_gemv_splitk_floats(int M, int N);
/* out[r] = LayerNorm(x[r]) bf16, r < m (nn.LayerNorm, _torch.py:62: norm_f for the backbone plugin),
 * with the GEMV LayerNorm prologue's arithmetic; k in {512, 1024, 2048, 4096}. */
int zmi_layernorm_rows(const void* x, int ldx, int m, int k, const void* w, const void* b, float eps, void* out,
                       int ldo, void* stream);

/* ---------------------------------------------------------------------------------------
 * Attention: GQA scaled-dot-product attention over the KV cache, one query position per
 * (query row). Replaces F.scaled_dot_product_attention(q, k, v, is_causal, enable_gqa)
 * at zonos/backbone/_torch.py:136 for decode (1 query) and prefill (causal = position bound).
 * ------------------------------------------------------------------------------------- */
/* K cache [rows][hkv][smax][hd], V cache transposed [rows][hkv][hd][smax] (bf16, as the QKV
 * epilogue writes them). q_kv_row may be NULL: query i then reads KV-cache row i (decode).
 * Softmax in the 512-key block structure of the reference's CPU kernel (probabilities rounded to
 * bf16 before P.V). Keys are processed in chunks of zmi_attention_chunk() keys whose partials go
 * to part_o [n_query*hkv][chunks][hq/hkv][hd] and part_lm [..][2] (zmi_attention_partial_floats
 * floats of o; 1/64 of that for lm), merged in-kernel by each query's last-arriving chunk.
 * `work` holds zmi_attention_work_bytes(...) zero-initialised bytes, re-armed by every launch; its
 * first 4 bytes become nonzero if a cross-chunk hand-off timed out. */
int zmi_attention(const void* q, int ldq, const void* k_cache, const void* v_cache, const int* q_kv_row,
                  const int* q_pos, int n_query, int hq, int hkv, int hd, int smax, int max_pos, void* out,
                  int ldo, float* part_o, float* part_lm, void* work, void* stream);
/* Same op with an explicit kernel choice: 0 = library choice (as zmi_attention), 1 = the chunked
 * kernel above (any length, one launch), 2 = the chunked kernel as two launches (scores and maxima, then the
 * rest: no workgroup waits on another), 3 = three launches (the merge as its own launch), 4 / 8 = the
 * whole-query kernel with that many output-dim slices per (query, kv head): every slice reads all of the
 * query's keys and no workgroup waits on another (max_pos < zmi_attention_max_keys_whole()). All variants
 * return identical bits. */
int zmi_attention_variant(const void* q, int ldq, const void* k_cache, const void* v_cache, const int* q_kv_row,
                          const int* q_pos, int n_query, int hq, int hkv, int hd, int smax, int max_pos, void* out,
                          int ldo, float* part_o, float* part_lm, void* work, int variant, void* stream);
int zmi_attention_max_keys_whole(void);
/* The kernel variant zmi_attention_variant / zmi_attention_pf run for `variant` (0 = library choice: 5, the
 * 512-key block form, from 32 (query, kv head) units, else 1, the chunked kernel); no launch. */
int zmi_attention_pick(int n_query, int hkv, int variant);
/* Fused decode block (reference _torch.py:114-136 for one decode step): the LayerNorm'd QKV
 * projection `qkv` (EPI_QKV arguments as for zmi_gemv_launch: M <= 16 rows, K = 2048, 4 query heads
 * per kv head, row_kv set) and the attention of every row at its position, in ONE launch whose
 * attention workgroups load the cached K / V while the projection streams its weights. q, the KV
 * cache writes and attn_out (bf16 [M][ldo]) are bit-identical to zmi_gemv_launch(QKV) followed by
 * zmi_attention. gran: zmi_attn_block_gran_words(M, hkv) u64 words of {value, tag = position + 1}
 * hand-off granules; a row's words must not hold tag pos + 1 from an earlier use when it runs at
 * position pos (zero them when a row starts a new utterance; consecutive steps need nothing).
 * err: set nonzero if a wait gave up (or a row's position exceeds the form's reach, see below).
 * slices: 4 or 8 workgroups per (row, kv head), optionally | ZMI_ATTNBLK_SELF:
 *   plain      the slices exchange scores (each scores 1/slices of the keys); positions < 1280;
 *   SELF       every slice scores all keys itself, nothing is exchanged between slices; positions < 1024;
 *   SPLIT      (slices 8) one workgroup per 128-key chunk: each reads only its chunk's K / V, the chunks
 *              exchange their maxima and P.V partials (two small hand-offs); positions < 1024.
 * zmi_attn_block_max_pos(slices) is the last position the form accepts; any smax is allowed (the engine
 * picks the form per step from the rows' positions). The projection's prologue is LayerNorm (pro AUTO with ln_w) or
 * ADDLN (pro ZMI_PRO_ADDLN: the hybrid's layer_norm_fn(hidden, residual), aux / ld_aux / res_out as for
 * zmi_gemv_launch). */
int zmi_attn_block(const ZmiGemvArgs* qkv, void* gran, unsigned* err, void* attn_out, int ldo, int slices,
                   void* stream);
enum { ZMI_ATTNBLK_SELF = 256, ZMI_ATTNBLK_SPLIT = 512 };
int zmi_attn_block_max_pos(int slices);
int64_t zmi_attn_block_gran_words(int rows, int hkv);
/* zmi_attn_block plus `blocks` prefetch-only workgroups that read ptr[0..1][0 .. bytes) once during the
 * attention phase (HBM is nearly idle there): the next launches' weights (out_proj, the head of fc1) are
 * then served from the Infinity Cache. Results are those of zmi_attn_block; `sink` is a scratch word the
 * prefetch may write (never read). */
typedef struct ZmiPrefetch {
  const void* ptr[2];
  int64_t bytes[2];
  unsigned* sink;
  int blocks, reserved;
} ZmiPrefetch;
int zmi_attn_block_pf(const ZmiGemvArgs* qkv, void* gran, unsigned* err, void* attn_out, int ldo, int slices,
                      const ZmiPrefetch* prefetch, void* stream);
/* zmi_attn_block_pf with the layer's out_proj in the same launch (the chunk-split forms: slices = 8 or 24 |
 * ZMI_ATTNBLK_SPLIT). With the LayerNorm prologue `oproj` holds the plain EPI_RESIDUAL GEMV arguments as for zmi_gemv_launch;
 * with the ADDLN prologue (the hybrid's MHA blocks) the role stores bf16(out_proj) to oproj->out (EPI_STORE: the hidden
 * rows the next block's add + LayerNorm reads; not the residual buffers). The LayerNorm case:
 * (W = out_proj weights, K = hq hd, N % 16 == 0, X = attn_out, out = the residual rows x, M = qkv->M), replacing
 * reference _torch.py:115,140 and the residual add :100. Its workgroups follow the attention ones: they load their
 * weight slice at their start and gather the attention output from the merging workgroups' {pair, tag} granules
 * (in the unit's granule area) once those workgroups' flags carry the row's tag, so no out_proj launch follows.
 * attn_out is still written. Results are bit-identical to zmi_attn_block_pf + zmi_gemv_launch(oproj). */
int zmi_attn_block_oproj(const ZmiGemvArgs* qkv, const ZmiGemvArgs* oproj, void* gran, unsigned* err, void* attn_out,
                         int ldo, int slices, const ZmiPrefetch* prefetch, void* stream);
/* zmi_attention_variant plus prefetch-only workgroups (variant 0 / 1: `prefetch->blocks` of them at the end
 * of the grid) that read prefetch->ptr[0..1][0 .. bytes) once, so the next launches (out_proj, the head of
 * fc1) find those weights in the Infinity Cache: they run on the CUs the chunks vacate, while the chunks
 * exchange maxima and merge (HBM nearly idle). prefetch may be NULL. Results are zmi_attention_variant's. */
int zmi_attention_pf(const void* q, int ldq, const void* k_cache, const void* v_cache, const int* q_kv_row,
                     const int* q_pos, int n_query, int hq, int hkv, int hd, int smax, int max_pos, void* out, int ldo,
                     float* part_o, float* part_lm, void* work, int variant, const ZmiPrefetch* prefetch,
                     void* stream);
int64_t zmi_attention_work_bytes(int n_query, int hq, int hkv, int hd, int max_pos);
int64_t zmi_attention_partial_floats(int n_query, int hq, int hkv, int hd, int max_pos);
int zmi_attention_chunk(void);

/* ---------------------------------------------------------------------------------------
 * Sampler + EOS state machine + delay-pattern frame write, per utterance slot.
 * Replaces model.py:112-115 (CFG), :266-267/280 (EOS logit bias), sampling.py:99-182
 * (repetition penalty, greedy / softmax / unified / top-p / top-k / min-p / exponential race)
 * and model.py:283-299 (EOS diagonal, masked_scatter_ frame compaction, counters).
 * ------------------------------------------------------------------------------------- */
typedef struct ZmiSampling {
  float temperature, top_p, min_p, linear, conf, quad, rep_penalty, cfg_scale;
  int top_k, rep_window;
  uint64_t seed;
} ZmiSampling;

typedef struct ZmiSlots {
  int* active;      /* [S] 1 while generating                                              */
  int* pos;         /* [S] tokens in the KV cache (= next position)                         */
  int* offset;      /* [S] last written delayed-frame index (reference `offset`)            */
  int* remaining;   /* [S] reference `remaining_steps`                                      */
  int* stopping;    /* [S] reference `stopping`                                             */
  int* step;        /* [S] decode steps done                                                */
  int* delayed;     /* [S][9][tcap] delayed codes (int32; -1 unknown, 1024 EOS, 1025 mask)   */
  const ZmiSampling* params; /* [S]                                                           */
  const int* total_len; /* [S] delayed length P + N + 9 (frames at or past it are not written) */
  int tcap;
  int n_slots;
} ZmiSlots;

/* mode 0 = decode step (bias + penalty + FSM), 1 = prefill (no bias, no penalty, no FSM).
 * With emb != NULL the slot's next input frame is embedded in the same launch (x[2s], x[2s+1],
 * model.py:97-98,142) and row_kv/row_pos (optional) receive the next step's KV row / position. */
int zmi_sample_step(const ZmiSlots* slots, const float* logits_rows, const float* noise, int* next_tokens,
                    unsigned* counters, int mode, int slot_begin, int slot_count, const void* emb, int d, void* x,
                    int* row_kv, int* row_pos, void* stream);
/* zmi_sample_step mode 0 for a launch whose slots all sample greedily (temperature <= 0; the caller
 * guarantees it): one workgroup per slot, no in-launch hand-off between codebooks; identical results. */
int zmi_sample_step_greedy(const ZmiSlots* slots, const float* logits_rows, int* next_tokens, int slot_begin,
                           int slot_count, const void* emb, int d, void* x, int* row_kv, int* row_pos, void* stream);
/* sample_from_logits (sampling.py:117-182) on its own: logits f32 [batch][9][1026] as given (no CFG,
 * no EOS bias), optional generated_tokens int32 [batch][9][gen_len] for the repetition penalty,
 * one parameter block (device), optional exponential noise [batch][9][1026]; tokens int32 [batch][9]. */
int zmi_sample_logits(const float* logits, const int* generated, int gen_len, int batch, const ZmiSampling* params,
                      const float* noise, int* tokens, void* stream);
/* apply_delay_pattern / revert_delay_pattern (codebook_pattern.py:5-12) on int64 [batch][9][T]
 * (apply: out [batch][9][T + 9]; revert: T >= 9, out [batch][9][T - 9]). */
int zmi_apply_delay_pattern(const int64_t* codes, int64_t* out, int batch, int T, int64_t mask_token, void* stream);
int zmi_revert_delay_pattern(const int64_t* codes, int64_t* out, int batch, int T, void* stream);
/* x[2s], x[2s+1] = sum_k emb_k[delayed[s][k][offset[s]]]  (model.py:97-98,142) and the
 * per-row (kv row, position) tables of the step (-1 position for inactive slots). */
int zmi_embed_step(const ZmiSlots* slots, const void* emb, int d, void* x, int* row_kv, int* row_pos,
                   void* stream);
/* prefill embedding rows: x[s] = sum_k emb_k[codes[k][s]] for s < n (model.py:195) */
int zmi_embed_codes(const int* codes, int ld_codes, int n, const void* emb, int d, void* x, int ldx, void* stream);
/* delayed[slot] = apply_delay_pattern(prefix codes | -1)    (codebook_pattern.py:5-7)      */
int zmi_delay_init(const ZmiSlots* slots, int slot, const int* prefix, int prefix_len, int total_len, void* stream);
/* out[9][T] int64 = revert_delay_pattern(delayed[slot]) with >=1024 -> 0 (model.py:309-311) */
int zmi_delay_revert(const ZmiSlots* slots, int slot, int64_t* out, int t_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * DAC 44.1 kHz decoder (DACAutoencoder.decode, autoencoder.py:25-27 -> transformers DacModel).
 * Activations are fp16, channels-last [T][C]; weights fp16 channel-blocked per tap [tap][Ci/32][Co][32] (one
 * 32-channel step of 16 output channels is 1 KiB contiguous: one LDS-DMA piece), except 1x1 convs (taps == 1):
 * [Co][Ci].
 * ------------------------------------------------------------------------------------- */
/* z[t][c] = sum_i (out_proj_i(codebook_i[codes[i][t]]))   (modeling_dac.py:347-371)          */
int zmi_dac_from_codes(const int64_t* codes, int T, const float* codebooks, const float* proj_w,
                       const float* proj_b, void* z, void* stream);
/* out[t_out][co] = epi( bias + sum_tap sum_ci W[tap][co][ci] * x[t_in][ci] ) with
 *   t_in = q + in_off + tap * tap_step, t_out = q * out_stride + out_phase, q in [0, n_out)
 * epilogue: + skip (fp16, optional), store raw (optional), snake(alpha) (optional) and/or the
 * raw fp32 value (optional, the encoder's latents). */
int zmi_dac_conv(const void* x, int t_in, int c_in, const void* w, const float* bias, int c_out, int taps,
                 int tap_step, int in_off, int n_out, int out_stride, int out_phase, int t_out, const void* skip,
                 void* out_raw, void* out_snake, const float* alpha, float* out_f32, void* stream);
/* DAC encode (DACAutoencoder.encode, autoencoder.py:22-23 -> DacModel.encode, modeling_dac.py:583-608).
 * col fp16 [T][32] = the 7 taps of encoder.conv1 around each sample (im2col, zero padded). */
int zmi_dac_im2col7(const float* wav, int t, void* col, void* stream);
/* residual VQ of latents f32 [T][1024] -> codes int64 [9][T] (modeling_dac.py:283-345, 123-173);
 * in_w [9][8][1024], in_b [9][8], codebooks [9][1024][8] raw and l2-normalised, codebooks_n2 =
 * |normalised row|^2 [9][1024], out_w [9][1024][8], out_b [9][1024]; all fp32. */
int zmi_dac_vq(const float* latents, int t, const float* in_w, const float* in_b, const float* codebooks,
               const float* codebooks_n, const float* codebooks_n2, const float* out_w, const float* out_b,
               int64_t* codes, void* stream);
/* polyphase ConvTranspose1d(c_in, c_out, k = 2 stride, stride, pad) of a DacDecoderBlock (modeling_dac.py:222-240),
 * every phase in one launch: w_phases fp16 [stride][2][c_in/32][c_out][32], phase rho's taps (rho + pad) % stride and
 * + stride, transposed; out [stride t_in][c_out] raw and / or Snake'd with alpha. */
int zmi_dac_conv_t(const void* x, int t_in, int c_in, const void* w_phases, const float* bias, int c_out, int stride,
                   int pad, void* out_raw, void* out_snake, const float* alpha, void* stream);
/* final Snake'd [T][c_in] -> conv k7 (c_in->1) -> tanh -> f32 [T]  (modeling_dac.py:438-441), on the
 * MFMA conv kernel: w_pad fp16 [7][c_in/32][32][32] (output channel 0 = the filter, 1..31 zero), bias_pad f32 [32]. */
int zmi_dac_conv_out(const void* x, int t, int c_in, const void* w_pad, const float* bias_pad, float* out,
                     void* stream);

/* ---------------------------------------------------------------------------------------
 * Prefix conditioner (Zonos.prepare_conditioning, model.py:204-212 -> PrefixConditioner.forward,
 * conditioning.py:300-310): one output row per conditioning token, then LayerNorm, bf16 out.
 * Each row names a parameter block and how to produce its d values before the LayerNorm.
 * ------------------------------------------------------------------------------------- */
enum {
  ZMI_COND_EMBED = 0,       /* table[index] (phoneme embedding :233, IntegerConditioner :270)      */
  ZMI_COND_VECTOR = 1,      /* table[0..d) (learned uncond_vector, conditioning.py:45-46)          */
  ZMI_COND_FOURIER = 2,     /* [cos f | sin f], f = 2 pi xn @ W^T (FourierConditioner :253-258)     */
  ZMI_COND_LINEAR = 3,      /* x @ W^T + b (PassthroughConditioner + projection "linear" :24-25)   */
  ZMI_COND_PASSTHROUGH = 4  /* x (PassthroughConditioner, projection "none")                      */
};
typedef struct ZmiCondParam {
  const void* table;   /* bf16 [rows][d] (EMBED) or [d] (VECTOR)                                */
  const void* weight;  /* bf16 [d/2][in_dim] (FOURIER) or [d][in_dim] (LINEAR)                  */
  const void* bias;    /* bf16 [d] (LINEAR) or NULL                                             */
  int in_dim;          /* input width (<= 256)                                                  */
  int pad;
  float min_val, max_val; /* FOURIER input normalisation                                         */
} ZmiCondParam;
typedef struct ZmiCondRow {
  int param;  /* index into the parameter array                                                 */
  int kind;   /* ZMI_COND_*                                                                      */
  int index;  /* EMBED row                                                                       */
  int x_off;  /* offset of this row's inputs in x (FOURIER / LINEAR / PASSTHROUGH)               */
} ZmiCondRow;
/* out[r][0..d) = LayerNorm(row r) for r < n_rows; params / rows / x are device arrays. */
int zmi_prefix_condition(const ZmiCondParam* params, const ZmiCondRow* rows, int n_rows, const float* x, int d,
                         const void* ln_w, const void* ln_b, float eps, void* out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Hybrid backbone (Zonos-v0.1-hybrid, zonos/backbone/_mamba_ssm.py:9-57): the blocks mamba-ssm
 * 2.2.4's create_block builds (Mamba2 mixer, MHA at attn_layer_idx, fused add + LayerNorm).
 * mamba-ssm is not in this image: parity unpinned (oracle/hybrid_cpu.py restates it).
 * ------------------------------------------------------------------------------------- */
typedef struct ZmiMamba2Args {
  const void* zxbcdt;   /* bf16 [M][ld_zx] in_proj output: z [d_ssm] | xBC [d_ssm + 2 d_state] | dt [nheads] */
  int ld_zx, M;
  int d_ssm, nheads, headdim, d_state, d_conv, ngroups; /* headdim 64, d_state 128, d_conv 4, ngroups 1 */
  const void* conv_w;   /* bf16 [d_ssm + 2 d_state][d_conv] depthwise conv1d weight                  */
  const void* conv_b;   /* bf16 [d_ssm + 2 d_state]                                                  */
  const float* dt_bias; /* f32 [nheads]                                                              */
  const float* A;       /* f32 [nheads] = -exp(A_log)                                                */
  const float* D;       /* f32 [nheads]                                                              */
  void* conv_ring;      /* bf16 [rows][d_conv][d_ssm + 2 d_state]: raw xBC of position q in slot q % 4 */
  void* ssm;            /* bf16 [rows][nheads][headdim][d_state]                                    */
  void* y;              /* bf16 [M][ldy] out: C.h + D x (before the gated norm)                      */
  int ldy, gz_g;        /* gz_g: 1 = gz receives g = y * gate (for ZMI_PRO_GRMS_G), 0 = the gate     */
  const int* row_pos;   /* [M] position of the row's token (< 0: inactive row; step only)           */
  const int* row_kv;    /* [M] state row of each activation row (NULL: row m)                       */
  float* gz;            /* step only, optional: f32 [M][ldy] the gate z * sigmoid(z) of RMSNormGated */
} ZmiMamba2Args;
/* Decode: causal_conv1d_update + SiLU + selective_state_update(dt_softplus) for one token per row
 * (mamba_ssm/modules/mamba2.py Mamba2.step). */
int zmi_mamba2_step(const ZmiMamba2Args* args, void* stream);
/* Prefill from an empty state: M / seq_len sequences of seq_len rows (causal_conv1d_fn +
 * mamba_chunk_scan_combined of Mamba2.forward), leaving each sequence's final state and conv ring. */
int zmi_mamba2_scan(const ZmiMamba2Args* args, int seq_len, void* stream);
/* The same prefill, parallel forms (the one HybridEngine runs): a conv + SiLU / dt launch into `ws`, then either
 * the state-space-dual matrix form (ZMI_OPT_SCAN_PQ 0, the default, sequences <= 256: y = (C B^T o decay) dt x on
 * MFMA, one workgroup for y and one for the final state per (sequence, head)) or the recurrence on PQ workgroups per
 * (sequence, head), fused multiply-adds (fp32 rounding differs from zmi_mamba2_scan's; all are checked against the
 * oracle). ws: >= zmi_mamba2_scan_ws_bytes(M, d_ssm, nheads). */
int zmi_mamba2_scan_ws(const ZmiMamba2Args* args, int seq_len, void* ws, int64_t ws_bytes, void* stream);
int64_t zmi_mamba2_scan_ws_bytes(int m, int d_ssm, int nheads);
/* layer_norm_fn(hidden, w, b, residual, prenorm=True): s = hidden + residual (fp32; hidden may be NULL:
 * s = residual), residual <- bf16(s) if store_residual, out = LayerNorm(s) bf16; k in {512 .. 4096}. */
int zmi_add_layernorm(const void* hidden, int ldh, void* residual, int ldr, int m, int k, const void* w,
                      const void* b, float eps, void* out, int ldo, int store_residual, void* stream);
/* RMSNormGated(norm_before_gate=False): out = rmsnorm(y * silu(z)) * w, bf16; k in {512 .. 4096}. */
int zmi_gated_rmsnorm(const void* y, int ldy, const void* z, int ldz, int m, int k, const void* w, float eps,
                      void* out, int ldo, void* stream);
/* Decode: the Mamba2 in_proj GEMV (ADDLN prologue, K = 2048) and zmi_mamba2_step in ONE launch: the step
 * workgroups load their state / conv-ring / conv-weight operands under the in_proj's weight stream and take
 * the in_proj output from {pair, tag = position + 1} granules (`gran`: zmi_mamba_block_gran_words(M,
 * d_in_proj) words, zeroed when a row starts an utterance); 1 <= M <= 16; bit-identical to the two
 * separate launches; *err becomes nonzero if a wait timed out. */
int zmi_mamba_block(const ZmiGemvArgs* in_proj, const ZmiMamba2Args* step, void* gran, unsigned* err, void* stream);
int64_t zmi_mamba_block_gran_words(int rows, int d_in_proj);
/* zmi_mamba_block plus `prefetch->blocks` prefetch-only workgroups (ZmiPrefetch, as zmi_attn_block_pf) that
 * read the given ranges (the layer's out_proj weights) once during the step phase; same results. */
int zmi_mamba_block_pf(const ZmiGemvArgs* in_proj, const ZmiMamba2Args* step, void* gran, unsigned* err,
                       const ZmiPrefetch* prefetch, void* stream);

/* ---------------------------------------------------------------------------------------
 * Synthetic weights: fill with the counter-based uniform stream of zonos_vibes_amd/synthetic.py
 * dtype 0 = bf16, 1 = f32.
 * ------------------------------------------------------------------------------------- */
int zmi_fill_uniform(void* dst, int64_t n, uint64_t key, float scale, float offset, int dtype, void* stream);

/* ---------------------------------------------------------------------------------------
 * hipGraph helpers: capture whatever the caller enqueues on `stream` between begin/end and
 * replay it. The decode step (~130 launches) is captured once per batch geometry.
 * ------------------------------------------------------------------------------------- */
int zmi_graph_begin(void* stream);
int zmi_graph_end(void* stream, void** graph_exec);
int zmi_graph_launch(void* graph_exec, int times, void* stream);
int zmi_graph_destroy(void* graph_exec);

const char* zmi_last_error(void);
/* ABI version, bumped whenever a weight layout or an option's meaning changes: 4 = channel-blocked DAC conv weights
 * [tap][ci / 32][co][32] (zmi_dac_conv / conv_t / conv_out) and the round-5 ZMI_OPT_GEMM_ROWS bits; 5 =
 * ZMI_OPT_XC_HANDOFF and zmi_xcd_dealing; 6 = ZMI_PRO_GRMS_G and ZmiMamba2Args.gz_g. Check it before packing weights (zonos_vibes_amd/_lib.py refuses a library
 * whose version differs). */
int zmi_version(void);
/* 1 if this device deals a launch's workgroups round-robin over its XCDs (blocks b and b + 8 on one XCD, 8
 * distinct XCDs), 0 if not, negative on a launch error (zmi_last_error). Runs a probe launch and waits for it:
 * call it outside graph capture. Hand-offs through an XCD's L2 (ZMI_OPT_XC_HANDOFF 0) rely on this; the engine
 * calls it once per process and sets ZMI_OPT_XC_HANDOFF to 1 otherwise. */
int zmi_xcd_dealing(void* stream);
/* Launch-geometry knobs of the library (process-wide; speed only, no option changes a result):
 *   ZMI_OPT_GEMV_SPREAD (default 1): single-tile GEMV launches reserve enough LDS per workgroup that the
 *   dispatcher spreads their workgroups evenly over the CUs instead of packing several onto one CU.
 *   ZMI_OPT_GEMM_ROWS (default 3): plain K = 2048 GEMVs over many rows run the many-row form (64 columns per
 *   workgroup, activation tiles DMA'd two ahead, one barrier per tile) where it measured faster than the
 *   32-column tile loop; 0 = always the tile loop; bit 1: the dense-pair MFMA forms of the many-row form and of
 *   zmi_gemv_splitk (16 real columns per MFMA instead of 8, same bits; 1 = the M8 forms).
 *   ZMI_OPT_GEMV_SPREAD > 1: at most that many single-tile GEMV workgroups per CU (an occupancy probe).
 *   ZMI_OPT_XC_HANDOFF (default 0): hand-offs between workgroups the grid places on one XCD (blocks 8 apart under
 *          the round-robin dealing zmi_xcd_dealing checks): the chunk-split fused attention block's chunk maxima,
 *          l / M_j and P.V partials inside a (row, kv head) unit, the block-form attention's block maxima and
 *          partials, and zmi_mamba_block's z / x granules for the step workgroups of their head. 0 = workgroup-scope
 *          stores that keep the lines in that XCD's L2, where the consumers' agent-scope polls read them; 1 =
 *          write-through (agent-scope) stores, correct whatever the dealing (set where zmi_xcd_dealing returns 0).
 *          Speed only: either gives the same bits.
 *   Options 3..9: reserved (knobs of the fused / persistent decode forms measured slower and removed in round 6;
 *          their sources are on the git branch diag-forms).
 *   ZMI_OPT_DAC_WIDE (default 1): DAC convs on 256-row time tiles (512-thread workgroups) when the output has at
 *          least ZMI_OPT_DAC_WIDE_MIN (default 256) 256-row x 32-channel units; 0 = always 128-row tiles, 2 = always
 *          256.
 *   ZMI_OPT_ATTNBLK_SPREAD (default 5): zmi_attn_block's workgroups reserve LDS so the launch spreads over the chip;
 *          bits 0-1 for the 8-chunk split / score-exchange / self forms, bits 2-3 for the 24-chunk split form:
 *          0 = no reserve, 1 = one workgroup per CU, 2 = at most two.
 *   ZMI_OPT_DAC_STAGE (default 29): DAC convs on the staged K loop (one barrier per 32-channel step x all taps, one
 *          512-thread workgroup per CU); bit 0 the k7 convs, bit 1 the 1x1 convs, bit 2 the transposed convs,
 *          bit 3 512-row time tiles for the k7 convs where their grid is large enough (256 otherwise), bit 4 the
 *          256-row forms with 4 dedicated loader waves (768 threads).
 *   ZMI_OPT_DAC_STAGE_MIN (default 128): the staged form only where its grid has at least this many workgroups.
 *   ZMI_OPT_SCAN_PQ (default 0): zmi_mamba2_scan_ws's form: 0 = the quadratic (SSD) form for sequences of up to
 *          256 positions (MFMA tiles of C B^T, the decay matrix and the state sum; longer sequences take PQ 4), else
 *          the recurrence on PQ workgroups per (sequence, head) (1, 2 or 4; each thread then owns 4 / PQ head dims x
 *          8 state columns).
 *   ZMI_OPT_SPLITK_WGS (default 256): zmi_gemv_splitk splits the rows into groups of 16-row tiles until its grid
 *          has about this many workgroups (each row group re-reads its segment's weights); 0 = one row group.
 *   ZMI_OPT_SPLITK_STAGE (default 1): zmi_gemv_splitk stages 2 (K segment 1024) or 4 (512) 16-row tiles per LDS
 *          buffer, so twice the activation bytes are in flight per CU (~132 KB of LDS); 0 = one tile per buffer. */
enum { ZMI_OPT_GEMV_SPREAD = 0, ZMI_OPT_GEMM_ROWS = 1, ZMI_OPT_XC_HANDOFF = 2, /* 3..9 reserved */
       ZMI_OPT_DAC_WIDE = 10, ZMI_OPT_DAC_WIDE_MIN = 11, ZMI_OPT_ATTNBLK_SPREAD = 12, ZMI_OPT_DAC_STAGE = 13,
       ZMI_OPT_DAC_STAGE_MIN = 14, ZMI_OPT_SCAN_PQ = 15, ZMI_OPT_SPLITK_WGS = 16, ZMI_OPT_SPLITK_STAGE = 17,
       ZMI_OPT_COUNT = 18 };
int zmi_set_option(int which, int value);
int zmi_get_option(int which);

#ifdef __cplusplus
}
#endif
#endif /* ZONOS_HIP_H */
