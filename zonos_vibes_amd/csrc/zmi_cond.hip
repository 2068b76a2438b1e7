// Prefix conditioner, gfx950: every conditioning row of Zonos.prepare_conditioning in one launch.
//
// Reference: zonos/conditioning.py PrefixConditioner.forward :300-310 (per-conditioner rows,
// concatenated along the sequence, then nn.LayerNorm), Conditioner.forward :43-50 (learned uncond
// vector, else apply_cond + project), EspeakPhonemeConditioner :219-235 (phoneme embedding),
// FourierConditioner :241-258, IntegerConditioner :261-270, PassthroughConditioner :273-279;
// zonos/model.py:204-212 (cond rows, then uncond rows). The model runs in bf16, so every
// reference tensor op rounds to bf16 at its output; this kernel rounds at the same points:
//   fourier : xn = bf16((x - min) / (max - min)); s = bf16(fp32(2 pi) * xn);
//             f[j] = bf16(sum_i s_i * W[j][i]) (fp32 sum over input dims in order);
//             out = [bf16(cos f) | bf16(sin f)]
//   linear  : out[j] = bf16(sum_i x_i * W[j][i] + b[j])   (nn.Linear, fp32 accumulation)
//   embed / integer / uncond vector / passthrough: copies of bf16 rows
// then LayerNorm over the row in fp32 (mean, then centred sum of squares; y = (x rstd - mean rstd)
// w + b), rounded to bf16. One workgroup per output row; rows are independent.
#include "zmi_common.h"
#include "zmi_kernels.h"

#include "zonos_hip.h"

namespace {

constexpr int NT = 256;
constexpr int MAXD = 4096;
constexpr int PER = MAXD / NT;

__global__ __launch_bounds__(NT) void cond_kernel(const ZmiCondParam* __restrict__ params,
                                                  const ZmiCondRow* __restrict__ rows, const float* __restrict__ xin,
                                                  int d, const bf16_t* __restrict__ ln_w, const bf16_t* __restrict__ ln_b,
                                                  float eps, bf16_t* __restrict__ out) {
  __shared__ float red[NT / 64];
  __shared__ float s_in[256];
  const int r = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const ZmiCondRow row = rows[r];
  const ZmiCondParam p = params[row.param];
  const int kind = row.kind;
  float v[PER];
  const int n_my = (d - t + NT - 1) / NT;  // elements j = t + i*NT owned by this thread

  if (kind == ZMI_COND_FOURIER || kind == ZMI_COND_LINEAR) {
    // stage the (few) input values in LDS, with the reference's input rounding
    for (int i = t; i < p.in_dim; i += NT) {
      float xv = xin[row.x_off + i];
      if (kind == ZMI_COND_FOURIER) {
        const float xn = bfround((xv - p.min_val) / (p.max_val - p.min_val));
        xv = bfround(6.2831855f * xn);
      }
      s_in[i] = xv;
    }
    __syncthreads();
  }
  const bf16_t* w = reinterpret_cast<const bf16_t*>(p.weight);
  const bf16_t* tab = reinterpret_cast<const bf16_t*>(p.table);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = 0.f;
    if (i >= n_my) continue;
    const int j = t + i * NT;
    float y = 0.f;
    switch (kind) {
      case ZMI_COND_EMBED:
        y = bf2f(tab[(size_t)row.index * d + j]);
        break;
      case ZMI_COND_VECTOR:
        y = bf2f(tab[j]);
        break;
      case ZMI_COND_PASSTHROUGH:
        y = bfround(xin[row.x_off + j]);
        break;
      case ZMI_COND_FOURIER: {
        const int h = d / 2, jj = j < h ? j : j - h;
        float f = 0.f;
        for (int k = 0; k < p.in_dim; ++k) f += s_in[k] * bf2f(w[(size_t)jj * p.in_dim + k]);
        f = bfround(f);
        y = bfround(j < h ? cosf(f) : sinf(f));
        break;
      }
      case ZMI_COND_LINEAR: {
        float acc = 0.f;
        const bf16_t* wr = w + (size_t)j * p.in_dim;
        for (int k = 0; k < p.in_dim; ++k) acc += bfround(s_in[k]) * bf2f(wr[k]);
        const bf16_t* b = reinterpret_cast<const bf16_t*>(p.bias);
        y = bfround(acc + (b ? bf2f(b[j]) : 0.f));
        break;
      }
      default:
        y = 0.f;
    }
    v[i] = y;
  }

  // LayerNorm over the row (two block reductions, fixed order)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (i < n_my) s += v[i];
  s = wave_sum(s);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const float mean = ((red[0] + red[1]) + red[2] + red[3]) / (float)d;
  __syncthreads();
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (i < n_my) {
      const float c = v[i] - mean;
      ss += c * c;
    }
  ss = wave_sum(ss);
  if (lane == 0) red[wave] = ss;
  __syncthreads();
  const float rstd = 1.0f / sqrtf(((red[0] + red[1]) + red[2] + red[3]) / (float)d + eps);
  const float nb = -mean * rstd;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (i < n_my) {
      const int j = t + i * NT;
      out[(size_t)r * d + j] = (bf16_t)f2bf((v[i] * rstd + nb) * bf2f(ln_w[j]) + bf2f(ln_b[j]));
    }
}

}  // namespace

extern "C" int zmi_prefix_condition(const ZmiCondParam* params, const ZmiCondRow* rows, int n_rows, const float* x,
                                    int d, const void* ln_w, const void* ln_b, float eps, void* out, void* stream) {
  if (d <= 0 || d > MAXD || (d & 1)) return zmi_fail_msg("prefix_condition: d must be even and <= 4096");
  if (n_rows <= 0) return 0;
  hipLaunchKernelGGL(cond_kernel, dim3(n_rows), dim3(NT), 0, (hipStream_t)stream, params, rows, x, d,
                     (const bf16_t*)ln_w, (const bf16_t*)ln_b, eps, (bf16_t*)out);
  ZMI_CHECK(hipGetLastError());
  return 0;
}
