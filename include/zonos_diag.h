/* zonos_diag.h -- the diagnostic library libzonos_diag.so (built only by `python -m zonos_vibes_amd.build --diag`).
 *
 * Fused and persistent decode forms that are bit-identical to the product plan but measured SLOWER on MI355X
 * (DESIGN.md §5, §5b): they are kept, with their tests (skipped when this library is absent) and timing tools,
 * as the record of those experiments, outside the shipped libzonos_hip.so. They link against libzonos_hip.so
 * (zmi_last_error, zmi_set_option and the ZMI_OPT_* knobs are the main library's) and take its argument blocks
 * (ZmiGemvArgs). Conventions as zonos_hip.h. */
#ifndef ZONOS_DIAG_H
#define ZONOS_DIAG_H
#include "zonos_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fused decode launch of a block's second half (reference _torch.py:100-101, 147-152 up to the SwiGLU):
 * out_proj (EPI_RESIDUAL: X = the attention rows, out = the residual rows x, updated in place) and fc1
 * (LayerNorm of the new x, packed SwiGLU weights [16384][2048], EPI_SWIGLU: out = h [M][8192]) in ONE
 * launch of 256 workgroups (one per CU; needs 256 CUs): each streams its fc1 weight slice while the
 * out_proj chain runs, and receives the new residual rows as {bf16 pair, tag = position + 1} granules
 * (`gran`: zmi_ffn_block_gran_words(M) u64 words, out_proj->row_pos set; zero a row's words when it
 * starts a new utterance). x and h are bit-identical to the two zmi_gemv_launch calls. 1 <= M <= 16;
 * *err becomes nonzero if a wait gave up. */
int zmi_ffn_block(const ZmiGemvArgs* out_proj, const ZmiGemvArgs* fc1, void* gran, unsigned* err, void* stream);
int64_t zmi_ffn_block_gran_words(int rows);
/* Fused decode launch of a block after its QKV projection (reference _torch.py:136 attention, :140 out_proj,
 * :100-101 residual + norm2, :147-152 fc1 + SwiGLU) for 1 <= M rows with M x hkv <= 8 and positions
 * <= zmi_attn_ffn_max_pos(): the chunk-split attention of zmi_attn_block over the KV cache (q, K / V as the
 * preceding zmi_gemv_launch(qkv, EPI_QKV) left them: `qkv` is that launch's argument block), then out_proj
 * (EPI_RESIDUAL, X = attn_out) and the LayerNorm'd fc1 (EPI_SWIGLU), in ONE launch of 256 workgroups (one
 * per CU; needs 256 CUs) whose weight streams run under the attention chain. attn_out (bf16 [M][ldo]), x and
 * h are bit-identical to zmi_attn_block(SPLIT) + zmi_ffn_block, i.e. to zmi_attention + two zmi_gemv_launch.
 * Granule areas of {value, tag = position + 1} words (zero a row's words when it starts a new utterance):
 * xgran zmi_attn_block_gran_words(M, hkv), ogran and rgran zmi_attn_ffn_gran_words(M) each (rgran may be
 * zmi_ffn_block's area). out_proj->row_pos = qkv->row_pos. *err becomes nonzero if a wait gave up. */
int zmi_attn_ffn_block(const ZmiGemvArgs* qkv, const ZmiGemvArgs* out_proj, const ZmiGemvArgs* fc1, void* xgran,
                       void* ogran, void* rgran, unsigned* err, void* attn_out, int ldo, void* stream);
int64_t zmi_attn_ffn_gran_words(int rows);
int zmi_attn_ffn_max_pos(void);
/* Persistent decode launch of a block's second half at batch 1 (reference _torch.py:100-101 out_proj +
 * residual, :101 norm2, :147-152 fc1 + SwiGLU + fc2, and the second residual add): 256 workgroups, one per CU
 * (needs 256 CUs), each streaming its slice of out_proj, fc1 and fc2 through an LDS ring (non-temporal
 * LDS-DMA) that runs ahead of the in-launch hand-offs ({value, tag = position + 1} granules in `gran`:
 * zmi_ffn_engine_gran_words(M) u64 words per layer; zero a row's words when it starts a new utterance).
 * x (bf16 [M][ldx]) is updated in place to x + out_proj(attn) + fc2(SwiGLU(fc1(norm2(.)))) bit-identically to
 * zmi_gemv_launch(out_proj, EPI_RESIDUAL), zmi_gemv_launch(fc1 with the norm2 LayerNorm, EPI_SWIGLU) and
 * zmi_gemv_launch(fc2, EPI_RESIDUAL); h (optional) receives the SwiGLU rows. d_model 2048, d_ff 8192 (packed
 * weights as zmi_pack_weight), 1 <= M <= 2. *err becomes nonzero if a wait gave up. diag: NULL, or u64
 * [256][16] phase stamps (s_memrealtime, diagnostics). */
typedef struct ZmiFfnEngineArgs {
  const void* w_out;    /* packed out_proj [2048][2048]                                       */
  const void* w_fc1;    /* packed fc1 [16384][2048] (ZMI_PACK_SWIGLU)                           */
  const void* w_fc2;    /* packed fc2 [2048][8192]                                              */
  const void* ln_w;     /* norm2 weight / bias, bf16 [2048]                                     */
  const void* ln_b;
  float eps;
  int M;
  const void* attn;     /* bf16 [M][ld_attn] attention output rows                              */
  void* x;              /* bf16 [M][ldx] residual rows, updated in place                        */
  void* h;              /* bf16 [M][ldh] SwiGLU rows, or NULL                                   */
  int ld_attn, ldx, ldh, reserved;
  const int* row_pos;   /* [M] positions (tags = position + 1)                                  */
  void* gran;
  unsigned* err;
  void* diag;
} ZmiFfnEngineArgs;
int zmi_ffn_engine(const ZmiFfnEngineArgs* args, void* stream);
int64_t zmi_ffn_engine_gran_words(int rows);
/* Persistent decode launch of one whole transformer block at batch 1 (reference _torch.py:136 attention, :140
 * out_proj + residual :100-101, norm2, :147-152 fc1 + SwiGLU + fc2 + residual), then the NEXT op on the new
 * residual rows: next = 0: LayerNorm (lnn) + QKV projection of layer L + 1 (:114-126: RoPE, K / V of the rows'
 * positions into k_next / v_next, q overwritten with the next layer's q); next = 1 (last layer): norm_f (lnn) +
 * the 9 heads (model.py:100-101) into logits f32 [M][9][1026]. The attention reads q and this layer's caches as the
 * previous launch (the QKV GEMV of layer 0, or the previous layer's engine) left them. 256 workgroups, one per CU
 * (needs 256 CUs), streaming every weight of the layer through per-wave LDS-DMA rings that run ahead of the
 * in-launch hand-offs ({value, tag = position + 1} granules in `gran`: zmi_layer_engine_gran_words(M) u64 words
 * per layer; zero them when the rows start a new utterance). Positions <= zmi_layer_engine_max_pos(). Every output
 * is bit-identical to zmi_attention + the zmi_gemv_launch plan (out_proj RESIDUAL, fc1 LayerNorm SWIGLU, fc2
 * RESIDUAL, next QKV / LOGITS with the LayerNorm prologue). attn_out (optional) receives the attention rows.
 * d_model 2048, d_ff 8192, 16 query / 4 kv heads of 128, 1 <= M <= 2 (row r caches into KV row r). */
typedef struct ZmiLayerEngineArgs {
  const void* w_out;    /* packed out_proj [2048][2048]                                         */
  const void* w_fc1;    /* packed fc1 [16384][2048] (ZMI_PACK_SWIGLU)                             */
  const void* w_fc2;    /* packed fc2 [2048][8192]                                                */
  const void* w_next;   /* packed QKV [3072][2048] of layer L + 1, or the heads [9248][2048]      */
  const void* ln2_w;    /* norm2, bf16 [2048]                                                     */
  const void* ln2_b;
  const void* lnn_w;    /* norm of layer L + 1, or norm_f                                         */
  const void* lnn_b;
  float eps;
  int M, smax, next;
  const int* row_pos;   /* [M] positions (tags = position + 1)                                    */
  void* x;              /* bf16 [M][2048] residual rows, updated in place                         */
  void* q;              /* bf16 [M][2048] this layer's q; the next layer's q on return (QKV)      */
  const void* k_cache;  /* this layer's K [M][4][smax][128] and V^T [M][4][128][smax]             */
  const void* v_cache;
  void* k_next;         /* the next layer's caches (next = 0)                                     */
  void* v_next;
  const float* rope;    /* (cos, sin) table as for zmi_gemv_launch (next = 0)                     */
  void* attn_out;       /* optional bf16 [M][2048]                                                */
  float* logits;        /* next = 1                                                               */
  void* gran;
  unsigned* err;
  void* diag;           /* NULL, or u64 [256][32] phase stamps (diagnostics)                      */
} ZmiLayerEngineArgs;
int zmi_layer_engine(const ZmiLayerEngineArgs* args, void* stream);
int64_t zmi_layer_engine_gran_words(int rows);
int zmi_layer_engine_max_pos(void);

#ifdef __cplusplus
}
#endif
#endif
