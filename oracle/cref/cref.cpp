// oracle/cref — C++/OpenMP restatement of the hot path: TEST INFRASTRUCTURE (full-size oracle for the GPU
// parity tests) and bench.py's CPU baseline (kind "port"). Never linked into the product.
//
// It restates, for the CPU (AVX2 + FMA + F16C, OpenMP over OMP_NUM_THREADS threads):
//   * the synthetic-weight hash of oracle/synth.py (bit-exact);
//   * the encoder / adaptor / CTC head of oracle/encoder.py + oracle/frontend.py, i.e. the reference's
//     /root/reference/fun_asr_gguf/model_definition.py:9-337 (EncoderExportWrapperPaddable, SenseVoiceEncoderSmall,
//     CorrectTransformerAdaptor, CTCHeadExportWrapper) in fp32 on a packed, register-blocked SGEMM;
//   * the Qwen3 decoder of oracle/qwen3.py (llama.cpp's qwen3 graph with ggml q8_0 x q8_0 numerics: activations
//     quantised per 32-block with the ggml reference quantiser, exact int8 block dots as ggml_vec_dot_q8_0_q8_0
//     computes them on AVX2 — sign/maddubs/madd — scaled by f32(dw)*f32(dx) and summed in f32; f16 KV cache).
// Parity of this file is pinned in tests/test_cref.py against the numpy oracle and the reference goldens.
#include <immintrin.h>
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------------------------------
// synthetic weights (oracle/synth.py spec)
uint32_t fnv1a32(const std::string& s) {
  uint32_t h = 0x811C9DC5u;
  for (unsigned char c : s) {
    h ^= c;
    h *= 0x01000193u;
  }
  return h;
}
inline uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
uint32_t tensor_key(const std::string& name, uint32_t seed) { return lowbias32(fnv1a32(name) ^ (seed * 0x9E3779B9u)); }

// elements [i0, i1) of tensor `name` (flat index i -> lowbias32(i ^ key))
void gen_range(const std::string& name, int64_t i0, int64_t i1, float scale, float offset, uint32_t seed, float* out) {
  const uint32_t key = tensor_key(name, seed);
#pragma omp parallel for schedule(static)
  for (int64_t i = i0; i < i1; ++i) {
    const uint32_t h = lowbias32((uint32_t)i ^ key);
    const float u = (float)(h >> 8) * 5.9604644775390625e-08f * 2.0f - 1.0f;
    float w = u * scale;
    if (offset != 0.0f) w = w + offset;
    out[i - i0] = w;
  }
}
std::vector<float> gen(const std::string& name, int64_t n, float scale, float offset, uint32_t seed) {
  std::vector<float> v(n);
  gen_range(name, 0, n, scale, offset, seed, v.data());
  return v;
}

inline float f16_round(float x) { return _cvtsh_ss(_cvtss_sh(x, _MM_FROUND_TO_NEAREST_INT)); }
inline uint16_t f16_bits(float x) { return _cvtss_sh(x, _MM_FROUND_TO_NEAREST_INT); }
inline float f16_val(uint16_t b) { return _cvtsh_ss(b); }

// ggml reference q8_0 quantiser (gguf/quants.py:378-393): d = amax/127, id = d ? 1/d : 0, q = roundf(x*id),
// d stored fp16 (kept here as its f32 value)
void quant_row_q8(const float* x, int K, int8_t* q, float* d) {
  for (int b = 0; b < K / 32; ++b) {
    float amax = 0.f;
    for (int j = 0; j < 32; ++j) amax = std::max(amax, std::fabs(x[b * 32 + j]));
    const float dd = amax / 127.0f;
    const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
    d[b] = f16_round(dd);
    for (int j = 0; j < 32; ++j) q[b * 32 + j] = (int8_t)roundf(x[b * 32 + j] * id);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// SGEMM  C[m][n] (+)= sum_k A[m][k] * B[n][k]   (both operands K-contiguous: x @ W.T of nn.Linear)
constexpr int MR = 6, NR = 16, KC = 256, MC = 96, NC = 192;

void pack_a(const float* A, int64_t lda, int mc, int kc, float* Ap) {
  for (int p = 0; p < mc; p += MR)
    for (int k = 0; k < kc; ++k)
      for (int r = 0; r < MR; ++r) *Ap++ = (p + r < mc) ? A[(int64_t)(p + r) * lda + k] : 0.f;
}
void pack_b(const float* B, int64_t ldb, int nc, int kc, float* Bp) {
  for (int p = 0; p < nc; p += NR) {
    float* dst = Bp + (int64_t)p * kc;
    for (int c = 0; c < NR; ++c) {
      if (p + c < nc) {
        const float* src = B + (int64_t)(p + c) * ldb;
        for (int k = 0; k < kc; ++k) dst[k * NR + c] = src[k];
      } else {
        for (int k = 0; k < kc; ++k) dst[k * NR + c] = 0.f;
      }
    }
  }
}

inline void micro_6x16(int kc, const float* Ap, const float* Bp, float* C, int64_t ldc, int mr, int nr, bool acc) {
  __m256 c[MR][2];
  for (int r = 0; r < MR; ++r) c[r][0] = c[r][1] = _mm256_setzero_ps();
  for (int k = 0; k < kc; ++k) {
    const __m256 b0 = _mm256_loadu_ps(Bp), b1 = _mm256_loadu_ps(Bp + 8);
#pragma GCC unroll 6
    for (int r = 0; r < MR; ++r) {
      const __m256 a = _mm256_broadcast_ss(Ap + r);
      c[r][0] = _mm256_fmadd_ps(a, b0, c[r][0]);
      c[r][1] = _mm256_fmadd_ps(a, b1, c[r][1]);
    }
    Ap += MR;
    Bp += NR;
  }
  if (mr == MR && nr == NR) {
    for (int r = 0; r < MR; ++r) {
      float* cp = C + r * ldc;
      if (acc) {
        c[r][0] = _mm256_add_ps(c[r][0], _mm256_loadu_ps(cp));
        c[r][1] = _mm256_add_ps(c[r][1], _mm256_loadu_ps(cp + 8));
      }
      _mm256_storeu_ps(cp, c[r][0]);
      _mm256_storeu_ps(cp + 8, c[r][1]);
    }
  } else {
    alignas(32) float t[MR][NR];
    for (int r = 0; r < MR; ++r) {
      _mm256_store_ps(t[r], c[r][0]);
      _mm256_store_ps(t[r] + 8, c[r][1]);
    }
    for (int r = 0; r < mr; ++r)
      for (int j = 0; j < nr; ++j) C[r * ldc + j] = acc ? C[r * ldc + j] + t[r][j] : t[r][j];
  }
}

struct Epi {
  const float* bias = nullptr;
  int relu = 0;
  const float* add = nullptr;  // residual [m][n] (ld_add); may alias C
  int64_t ld_add = 0;
  const float* add2 = nullptr;
  int64_t ld_add2 = 0;
  float scale = 1.f;  // applied to the product before bias
};

void sgemm(int M, int N, int K, const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
           const Epi& e = Epi()) {
  const int nmb = (M + MC - 1) / MC, nnb = (N + NC - 1) / NC;
#pragma omp parallel
  {
    std::vector<float> Ap((size_t)MC * KC), Bp((size_t)NC * KC);
#pragma omp for collapse(2) schedule(dynamic)
    for (int nb = 0; nb < nnb; ++nb)
      for (int mb = 0; mb < nmb; ++mb) {
        const int n0 = nb * NC, m0 = mb * MC;
        const int nc = std::min(NC, N - n0), mc = std::min(MC, M - m0);
        for (int k0 = 0; k0 < K; k0 += KC) {
          const int kc = std::min(KC, K - k0);
          pack_a(A + (int64_t)m0 * lda + k0, lda, mc, kc, Ap.data());
          pack_b(B + (int64_t)n0 * ldb + k0, ldb, nc, kc, Bp.data());
          for (int j = 0; j < nc; j += NR)
            for (int i = 0; i < mc; i += MR)
              micro_6x16(kc, Ap.data() + (int64_t)i * kc, Bp.data() + (int64_t)j * kc, C + (int64_t)(m0 + i) * ldc + n0 + j,
                         ldc, std::min(MR, mc - i), std::min(NR, nc - j), k0 > 0);
        }
        for (int i = 0; i < mc; ++i) {
          float* c = C + (int64_t)(m0 + i) * ldc + n0;
          for (int j = 0; j < nc; ++j) {
            float y = c[j];
            if (e.scale != 1.f) y = y * e.scale;
            if (e.bias) y = y + e.bias[n0 + j];
            if (e.relu) y = std::max(y, 0.f);
            if (e.add2) y = y + e.add2[(int64_t)(m0 + i) * e.ld_add2 + n0 + j];  // (x W^T + b) + mem
            if (e.add) y = e.add[(int64_t)(m0 + i) * e.ld_add + n0 + j] + y;     // residual + (...)
            c[j] = y;
          }
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// encoder (oracle/encoder.py)
struct EncCfg {
  int n_mels, lfr_m, lfr_n, d_in, d_model, n_heads, d_ffn, n_blocks, n_tp_blocks, fsmn_k;
  int d_llm, adaptor_ffn, adaptor_blocks, adaptor_heads, ctc_blocks, ctc_heads, ctc_ffn, ctc_vocab;
};
struct Lin {
  std::vector<float> w, b;
  int n_in = 0, n_out = 0;
};
struct LN {
  std::vector<float> w, b;
};
struct Sanm {
  LN ln1, ln2;
  Lin qkv, out, w1, w2;
  std::vector<float> fsmn;  // [d][k]
  int d_in;
};
struct AdBlock {
  LN ln1, ln2;
  Lin q, k, v, o, w1, w2;
};
struct Adaptor {
  Lin l1, l2;
  std::vector<AdBlock> blocks;
};

struct Encoder {
  EncCfg c;
  uint32_t seed;
  std::vector<Sanm> blocks;
  LN after, tp;
  Adaptor ad, ctc;
  Lin ctc_lo;
  std::vector<float> basis, fbank;  // [402][400] (cos, -sin interleaved rows), [80][201]

  Lin lin(const std::string& p, int n_in, int n_out, bool bias = true) {
    Lin l;
    l.n_in = n_in;
    l.n_out = n_out;
    l.w = gen(p + ".weight", (int64_t)n_in * n_out, (float)std::sqrt(3.0 / n_in), 0.f, seed);
    if (bias) l.b = gen(p + ".bias", n_out, 0.02f, 0.f, seed);
    return l;
  }
  LN ln(const std::string& p, int d) { return LN{gen(p + ".weight", d, 0.1f, 1.0f, seed), gen(p + ".bias", d, 0.02f, 0.f, seed)}; }
  Sanm sanm(const std::string& p, int d_in) {
    const int d = c.d_model;
    Sanm s;
    s.d_in = d_in;
    s.ln1 = ln(p + ".norm1", d_in);
    s.ln2 = ln(p + ".norm2", d);
    s.qkv = lin(p + ".self_attn.linear_q_k_v", d_in, 3 * d);
    s.out = lin(p + ".self_attn.linear_out", d, d);
    s.fsmn = gen(p + ".self_attn.fsmn_block.weight", (int64_t)d * c.fsmn_k, (float)(std::sqrt(3.0 / c.fsmn_k) * 0.5), 0.f, seed);
    s.w1 = lin(p + ".feed_forward.w_1", d, c.d_ffn);
    s.w2 = lin(p + ".feed_forward.w_2", c.d_ffn, d);
    return s;
  }
  Adaptor adaptor(const std::string& p, int d_enc, int d_out, int d_ffn, int n_blocks) {
    Adaptor a;
    a.l1 = lin(p + ".linear1", d_enc, d_ffn);
    a.l2 = lin(p + ".linear2", d_ffn, d_out);
    for (int b = 0; b < n_blocks; ++b) {
      const std::string q = p + ".blocks." + std::to_string(b);
      AdBlock k;
      k.q = lin(q + ".self_attn.linear_q", d_out, d_out);
      k.k = lin(q + ".self_attn.linear_k", d_out, d_out);
      k.v = lin(q + ".self_attn.linear_v", d_out, d_out);
      k.o = lin(q + ".self_attn.linear_out", d_out, d_out);
      k.w1 = lin(q + ".feed_forward.w_1", d_out, d_out / 4);
      k.w2 = lin(q + ".feed_forward.w_2", d_out / 4, d_out);
      k.ln1 = ln(q + ".norm1", d_out);
      k.ln2 = ln(q + ".norm2", d_out);
      a.blocks.push_back(std::move(k));
    }
    return a;
  }

  static std::vector<float> linspace_f32(float start, float end, int steps) {
    std::vector<float> o(steps);
    const float step = (end - start) / (float)(steps - 1);
    const int half = steps / 2;
    for (int i = 0; i < steps; ++i) o[i] = i < half ? start + step * (float)i : end - step * (float)(steps - i - 1);
    return o;
  }

  Encoder(const EncCfg& cfg, uint32_t sd) : c(cfg), seed(sd) {
    blocks.push_back(sanm("audio_encoder.encoders0.0", c.d_in));
    for (int i = 0; i < c.n_blocks - 1; ++i) blocks.push_back(sanm("audio_encoder.encoders." + std::to_string(i), c.d_model));
    for (int i = 0; i < c.n_tp_blocks; ++i) blocks.push_back(sanm("audio_encoder.tp_encoders." + std::to_string(i), c.d_model));
    after = ln("audio_encoder.after_norm", c.d_model);
    tp = ln("audio_encoder.tp_norm", c.d_model);
    ad = adaptor("audio_adaptor", c.d_model, c.d_llm, c.adaptor_ffn, c.adaptor_blocks);
    ctc = adaptor("ctc_decoder", c.d_model, c.d_model, c.ctc_ffn, c.ctc_blocks);
    ctc_lo = lin("ctc_proj.ctc_lo", c.d_model, c.ctc_vocab);
    // STFT basis (frontend.stft_basis): periodic Hamming window, f32 phase 2*pi*f*t/400
    const double PI = 3.14159265358979323846;
    std::vector<float> win(400);
    const float wstep = (float)(2.0 * PI / 400.0);
    for (int n = 0; n < 400; ++n) win[n] = (float)std::cos((double)((float)n * wstep)) * -0.46f + 0.54f;
    basis.assign(402 * 400, 0.f);
    const float twopi = (float)(2.0 * PI);
    for (int f = 0; f < 201; ++f)
      for (int t = 0; t < 400; ++t) {
        const float om = ((twopi * (float)f) * (float)t) / 400.0f;
        basis[(2 * f) * 400 + t] = (float)std::cos((double)om) * win[t];
        basis[(2 * f + 1) * 400 + t] = -(float)std::sin((double)om) * win[t];
      }
    // HTK mel filterbank (frontend.mel_fbank)
    std::vector<float> allf = linspace_f32(0.f, 8000.f, 201);
    const double mmin = 2595.0 * std::log10(1.0 + 20.0 / 700.0), mmax = 2595.0 * std::log10(1.0 + 8000.0 / 700.0);
    std::vector<float> mp = linspace_f32((float)mmin, (float)mmax, 82), fp(82);
    for (int i = 0; i < 82; ++i) fp[i] = 700.0f * ((float)std::pow(10.0, (double)(mp[i] / 2595.0f)) - 1.0f);
    fbank.assign(80 * 201, 0.f);
    for (int j = 0; j < 201; ++j)
      for (int i = 0; i < 80; ++i) {
        const float fd0 = fp[i + 1] - fp[i], fd1 = fp[i + 2] - fp[i + 1];
        const float down = (-1.0f * (fp[i] - allf[j])) / fd0;
        const float up = (fp[i + 2] - allf[j]) / fd1;
        fbank[i * 201 + j] = std::max(0.0f, std::min(down, up));
      }
  }

  static void layer_norm(const float* x, int64_t ldx, float* y, int64_t ldy, int T, int D, const LN& p, double eps) {
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; ++t) {
      const float* r = x + (int64_t)t * ldx;
      double mu = 0, var = 0;
      for (int i = 0; i < D; ++i) mu += r[i];
      mu /= D;
      for (int i = 0; i < D; ++i) var += (r[i] - mu) * (r[i] - mu);
      var /= D;
      const double is = 1.0 / std::sqrt(var + eps);
      float* o = y + (int64_t)t * ldy;
      for (int i = 0; i < D; ++i) o[i] = (float)(((r[i] - mu) * is) * p.w[i] + p.b[i]);
    }
  }

  static void linear(const float* x, int64_t ldx, const Lin& l, float* y, int64_t ldy, int T, int relu = 0,
                     const float* add = nullptr, int64_t ld_add = 0, const float* add2 = nullptr, int64_t ld_add2 = 0) {
    Epi e;
    e.bias = l.b.empty() ? nullptr : l.b.data();
    e.relu = relu;
    e.add = add;
    e.ld_add = ld_add;
    e.add2 = add2;
    e.ld_add2 = ld_add2;
    if (add == y || add2 == y) {  // the GEMM stores partial products into C before the epilogue reads the residual
      std::vector<float> tmp((size_t)T * l.n_out);
      sgemm(T, l.n_out, l.n_in, x, ldx, l.w.data(), l.n_in, tmp.data(), l.n_out, e);
      for (int t = 0; t < T; ++t) std::memcpy(y + (int64_t)t * ldy, tmp.data() + (size_t)t * l.n_out, (size_t)l.n_out * 4);
      return;
    }
    sgemm(T, l.n_out, l.n_in, x, ldx, l.w.data(), l.n_in, y, ldy, e);
  }

  // softmax(q d^-0.5 @ k^T + (m - 1) 1e4) @ v per head; q/k/v strided [T][ld], out [T][ldo]
  static void attention(const float* q, const float* k, const float* v, int64_t ld, float* out, int64_t ldo, int T,
                        int H, int dk, const float* mask) {
    std::vector<float> qs((size_t)T * dk), S((size_t)T * T), vt((size_t)dk * T);
    const float scale = (float)std::pow((double)dk, -0.5);
    for (int h = 0; h < H; ++h) {
#pragma omp parallel for schedule(static)
      for (int t = 0; t < T; ++t)
        for (int i = 0; i < dk; ++i) {
          qs[(size_t)t * dk + i] = q[(int64_t)t * ld + h * dk + i] * scale;
          vt[(size_t)i * T + t] = v[(int64_t)t * ld + h * dk + i];
        }
      sgemm(T, T, dk, qs.data(), dk, k + h * dk, ld, S.data(), T);
#pragma omp parallel for schedule(static)
      for (int t = 0; t < T; ++t) {
        float* s = S.data() + (size_t)t * T;
        float mx = -INFINITY;
        for (int j = 0; j < T; ++j) {
          if (mask) s[j] = s[j] + (mask[j] - 1.0f) * 10000.0f;
          mx = std::max(mx, s[j]);
        }
        double z = 0;
        for (int j = 0; j < T; ++j) {
          s[j] = std::exp(s[j] - mx);
          z += s[j];
        }
        const float iz = (float)z;
        for (int j = 0; j < T; ++j) s[j] = s[j] / iz;
      }
      sgemm(T, dk, T, S.data(), T, vt.data(), T, out + h * dk, ldo);
    }
  }

  void sanm_block(std::vector<float>& x, const Sanm& w, int T, const float* m, bool first, std::vector<float>& buf) {
    const int d = c.d_model, din = w.d_in, K = c.fsmn_k;
    std::vector<float> h((size_t)T * din), qkv((size_t)T * 3 * d), mem((size_t)T * d), att((size_t)T * d);
    layer_norm(x.data(), din, h.data(), din, T, din, w.ln1, 1e-5);
    linear(h.data(), din, w.qkv, qkv.data(), 3 * d, T);
    // FSMN (oracle.encoder.fsmn): depthwise conv k=11 of v*m (zero pad 5/5) + v*m
    const int lp = (K - 1) / 2;
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; ++t)
      for (int ch = 0; ch < d; ++ch) {
        float o = 0.f;
        for (int j = 0; j < K; ++j) {
          const int tt = t + j - lp;
          if (tt < 0 || tt >= T) continue;
          o = o + (qkv[(size_t)tt * 3 * d + 2 * d + ch] * m[tt]) * w.fsmn[(size_t)ch * K + j];
        }
        mem[(size_t)t * d + ch] = o + qkv[(size_t)t * 3 * d + 2 * d + ch] * m[t];
      }
    attention(qkv.data(), qkv.data() + d, qkv.data() + 2 * d, 3 * d, att.data(), d, T, c.n_heads, d / c.n_heads, m);
    if (first) {
      x.assign((size_t)T * d, 0.f);
      linear(att.data(), d, w.out, x.data(), d, T, 0, nullptr, 0, mem.data(), d);
      return;
    }
    linear(att.data(), d, w.out, x.data(), d, T, 0, x.data(), d, mem.data(), d);
    std::vector<float> f((size_t)T * c.d_ffn);
    layer_norm(x.data(), d, h.data(), d, T, d, w.ln2, 1e-5);
    linear(h.data(), d, w.w1, f.data(), c.d_ffn, T, 1);
    linear(f.data(), c.d_ffn, w.w2, x.data(), d, T, 0, x.data(), d);
    (void)buf;
  }

  std::vector<float> run_adaptor(const Adaptor& a, const std::vector<float>& in, int d_enc, int d_out, int d_ffn,
                                 int H, int T, const float* mask) {
    std::vector<float> f((size_t)T * std::max(d_ffn, d_out)), x((size_t)T * d_out), h((size_t)T * d_out);
    std::vector<float> q((size_t)T * d_out), k((size_t)T * d_out), v((size_t)T * d_out), att((size_t)T * d_out);
    linear(in.data(), d_enc, a.l1, f.data(), d_ffn, T, 1);
    linear(f.data(), d_ffn, a.l2, x.data(), d_out, T);
    for (const AdBlock& b : a.blocks) {
      layer_norm(x.data(), d_out, h.data(), d_out, T, d_out, b.ln1, 1e-12);
      linear(h.data(), d_out, b.q, q.data(), d_out, T);
      linear(h.data(), d_out, b.k, k.data(), d_out, T);
      linear(h.data(), d_out, b.v, v.data(), d_out, T);
      // three separate [T][d] tensors: attention takes one stride, so interleave-free per-head GEMMs
      attention_sep(q.data(), k.data(), v.data(), d_out, att.data(), d_out, T, H, d_out / H, mask);
      linear(att.data(), d_out, b.o, x.data(), d_out, T, 0, x.data(), d_out);
      layer_norm(x.data(), d_out, h.data(), d_out, T, d_out, b.ln2, 1e-12);
      linear(h.data(), d_out, b.w1, f.data(), d_out / 4, T, 1);
      linear(f.data(), d_out / 4, b.w2, x.data(), d_out, T, 0, x.data(), d_out);
    }
    return x;
  }
  static void attention_sep(const float* q, const float* k, const float* v, int64_t ld, float* out, int64_t ldo, int T,
                            int H, int dk, const float* mask) {
    attention(q, k, v, ld, out, ldo, T, H, dk, mask);  // same strides for q, k, v
  }

  // one clip: audio [n_phys] with `valid` samples. Outputs enc [T][512], adaptor [T][d_llm] (rows >= target_len
  // zeroed), CTC ids [T] and top-1/top-2 logit margins [T]. Returns T = t_lfr_phys; *tgt = target_len.
  int forward(const float* audio, int64_t n_phys, int64_t valid, float* enc_out, float* ad_out, int32_t* ids_out,
              float* margin_out, int32_t* tgt_out) {
    const int t_phys = (int)(n_phys / 160 + 1), t_mel_valid = (int)(valid / 160 + 1);
    const int t_lfr_valid = (t_mel_valid + 5) / 6, T = (t_phys + 5) / 6;
    const int o1 = 1 + (t_lfr_valid - 3 + 2) / 2;
    const int tgt = (1 + (o1 - 3 + 2) / 2 - 1) / 2 + 1;
    // F1 mean removal over valid samples, pre-emphasis, mask
    double sum = 0;
    for (int64_t i = 0; i < valid; ++i) sum += audio[i];
    const float mean = (float)(sum / (double)valid);
    std::vector<float> a(n_phys), pre(n_phys);
    for (int64_t i = 0; i < n_phys; ++i) a[i] = i < valid ? (audio[i] - mean) * 1.0f : 0.f;
    for (int64_t i = 0; i < n_phys; ++i) {
      const float b = i == 0 ? a[0] : a[i] - 0.97f * a[i - 1];
      pre[i] = i < valid ? b : 0.f;
    }
    // F2/F3: frames of the 200/200 zero-padded signal, DFT GEMM, power, mel, log
    std::vector<float> frames((size_t)t_phys * 400), spec((size_t)t_phys * 402), power((size_t)t_phys * 201),
        mel((size_t)t_phys * 80);
#pragma omp parallel for schedule(static)
    for (int t = 0; t < t_phys; ++t)
      for (int j = 0; j < 400; ++j) {
        const int64_t s = (int64_t)t * 160 + j - 200;
        frames[(size_t)t * 400 + j] = (s >= 0 && s < n_phys) ? pre[s] : 0.f;
      }
    sgemm(t_phys, 402, 400, frames.data(), 400, basis.data(), 400, spec.data(), 402);
    for (size_t t = 0; t < (size_t)t_phys; ++t)
      for (int f = 0; f < 201; ++f) {
        const float re = spec[t * 402 + 2 * f], im = spec[t * 402 + 2 * f + 1];
        power[t * 201 + f] = re * re + im * im;
      }
    sgemm(t_phys, 80, 201, power.data(), 201, fbank.data(), 201, mel.data(), 80);
    for (auto& v : mel) v = std::log(v + 1e-7f);
    // F4 LFR (replicate padding), mask, x*sqrt(512) + PE (positions 1..T)
    const int D = c.d_in, half = D / 2;
    std::vector<float> x((size_t)T * D), m(T);
    const float inc = (float)std::log(10000.0f) / (float)(D / 2.0 - 1.0);
    std::vector<float> inv(half);
    for (int i = 0; i < half; ++i) inv[i] = (float)std::exp((double)((float)i * -inc));
    for (int t = 0; t < T; ++t) {
      m[t] = t < t_lfr_valid ? 1.f : 0.f;
      for (int s = 0; s < 7; ++s) {
        int src = t * 6 + s - 3;  // padded index minus the 3 left replicas
        src = std::max(0, std::min(src, t_phys - 1));
        src = std::min(src, t_mel_valid - 1);
        for (int b = 0; b < 80; ++b) x[(size_t)t * D + s * 80 + b] = mel[(size_t)src * 80 + b] * m[t];
      }
      for (int i = 0; i < half; ++i) {
        const float st = (float)(t + 1) * inv[i];
        float* r = x.data() + (size_t)t * D;
        r[i] = r[i] * 22.627416997969522f + (float)std::sin((double)st);
        r[half + i] = r[half + i] * 22.627416997969522f + (float)std::cos((double)st);
      }
    }
    // SenseVoiceEncoderSmall
    std::vector<float> buf;
    const int d = c.d_model;
    sanm_block(x, blocks[0], T, m.data(), true, buf);
    for (int i = 1; i < c.n_blocks; ++i) sanm_block(x, blocks[i], T, m.data(), false, buf);
    layer_norm(x.data(), d, x.data(), d, T, d, after, 1e-5);
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < d; ++i) x[(size_t)t * d + i] *= m[t];
    for (int i = 0; i < c.n_tp_blocks; ++i) sanm_block(x, blocks[c.n_blocks + i], T, m.data(), false, buf);
    layer_norm(x.data(), d, x.data(), d, T, d, tp, 1e-5);
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < d; ++i) x[(size_t)t * d + i] *= m[t];
    if (enc_out) std::memcpy(enc_out, x.data(), (size_t)T * d * 4);
    // adaptor (key mask m), rows >= target_len zeroed (model_definition.py:317-321)
    if (ad_out) {
      std::vector<float> y = run_adaptor(ad, x, d, c.d_llm, c.adaptor_ffn, c.adaptor_heads, T, m.data());
      for (int t = 0; t < T; ++t)
        for (int i = 0; i < c.d_llm; ++i) ad_out[(size_t)t * c.d_llm + i] = t < tgt ? y[(size_t)t * c.d_llm + i] : 0.f;
    }
    // CTC head, unmasked (model_definition.py:336), projection in vocab chunks with a running top-2
    if (ids_out) {
      std::vector<float> h = run_adaptor(ctc, x, d, d, c.ctc_ffn, c.ctc_heads, T, nullptr);
      const int CH = 4096;
      std::vector<float> lg((size_t)T * CH), b1(T, -INFINITY), b2(T, -INFINITY);
      std::vector<int> i1(T, 0);
      for (int n0 = 0; n0 < c.ctc_vocab; n0 += CH) {
        const int nc = std::min(CH, c.ctc_vocab - n0);
        Epi e;
        e.bias = ctc_lo.b.data() + n0;
        sgemm(T, nc, d, h.data(), d, ctc_lo.w.data() + (size_t)n0 * d, d, lg.data(), nc, e);
#pragma omp parallel for schedule(static)
        for (int t = 0; t < T; ++t)
          for (int j = 0; j < nc; ++j) {
            const float v = lg[(size_t)t * nc + j];
            if (v > b1[t]) {
              b2[t] = b1[t];
              b1[t] = v;
              i1[t] = n0 + j;
            } else if (v > b2[t]) {
              b2[t] = v;
            }
          }
      }
      for (int t = 0; t < T; ++t) {
        ids_out[t] = i1[t];
        if (margin_out) margin_out[t] = b1[t] - b2[t];
      }
    }
    if (tgt_out) *tgt_out = tgt;
    return T;
  }
};

// ---------------------------------------------------------------------------------------------------------------
// Qwen3 q8_0 decoder (oracle/qwen3.py)
struct Q8 {
  int O = 0, K = 0;
  std::vector<int8_t> q;
  std::vector<float> d;  // f32 value of the fp16 scale
};
struct LlmLayer {
  Q8 wq, wk, wv, wo, gate, up, down;
  std::vector<float> attn_norm, ffn_norm, q_norm, k_norm;
};

// ggml_vec_dot_q8_0_q8_0 on AVX2: per block |w| (x) sign(a, w), maddubs -> madd -> f32, scaled by dw*da, summed
// across blocks in 8 f32 lanes, then a horizontal sum
inline float dot_q8(const int8_t* wq, const float* wd, const int8_t* aq, const float* ad, int nb) {
  __m256 acc = _mm256_setzero_ps();
  const __m256i ones = _mm256_set1_epi16(1);
  for (int b = 0; b < nb; ++b) {
    const __m256i w = _mm256_loadu_si256((const __m256i*)(wq + 32 * b));
    const __m256i a = _mm256_loadu_si256((const __m256i*)(aq + 32 * b));
    const __m256i p16 = _mm256_maddubs_epi16(_mm256_sign_epi8(w, w), _mm256_sign_epi8(a, w));
    const __m256 p = _mm256_cvtepi32_ps(_mm256_madd_epi16(p16, ones));
    acc = _mm256_fmadd_ps(_mm256_set1_ps(wd[b] * ad[b]), p, acc);
  }
  __m128 s = _mm_add_ps(_mm256_castps256_ps128(acc), _mm256_extractf128_ps(acc, 1));
  s = _mm_add_ps(s, _mm_movehl_ps(s, s));
  s = _mm_add_ss(s, _mm_movehdup_ps(s));
  return _mm_cvtss_f32(s);
}

struct Llm {
  int L, E, H, KV, Dh, F, V, n_ctx, max_seqs;
  float theta, eps;
  uint32_t seed;
  Q8 tok;
  std::vector<LlmLayer> layers;
  std::vector<float> out_norm, rcos, rsin;
  std::vector<uint16_t> kc, vc;  // [seq][layer][n_ctx][KV*Dh] fp16

  Q8 q8(const std::string& name, int O, int K, float scale) {
    Q8 m;
    m.O = O;
    m.K = K;
    m.q.resize((size_t)O * K);
    m.d.resize((size_t)O * K / 32);
    const int64_t chunk = 1 << 22;  // generate + quantise 4M values at a time
    std::vector<float> tmp(chunk);
    for (int64_t i0 = 0; i0 < (int64_t)O * K; i0 += chunk) {
      const int64_t i1 = std::min<int64_t>((int64_t)O * K, i0 + chunk);
      gen_range(name, i0, i1, scale, 0.f, seed, tmp.data());
      const int64_t rows = (i1 - i0) / K;
#pragma omp parallel for schedule(static)
      for (int64_t r = 0; r < rows; ++r)
        quant_row_q8(tmp.data() + r * K, K, m.q.data() + i0 + r * K, m.d.data() + (i0 + r * K) / 32);
    }
    return m;
  }

  Llm(const int32_t* cfg, float rope_theta, float rms_eps, int nctx, int mseqs, uint32_t sd)
      : L(cfg[0]), E(cfg[1]), H(cfg[2]), KV(cfg[3]), Dh(cfg[4]), F(cfg[5]), V(cfg[6]), n_ctx(nctx), max_seqs(mseqs),
        theta(rope_theta), eps(rms_eps), seed(sd) {
    auto s = [](int n_in) { return (float)std::sqrt(3.0 / n_in); };
    tok = q8("token_embd.weight", V, E, 0.05f);
    for (int l = 0; l < L; ++l) {
      const std::string b = "blk." + std::to_string(l) + ".";
      LlmLayer w;
      w.attn_norm = gen(b + "attn_norm.weight", E, 0.1f, 1.0f, seed);
      w.wq = q8(b + "attn_q.weight", H * Dh, E, s(E));
      w.wk = q8(b + "attn_k.weight", KV * Dh, E, s(E));
      w.wv = q8(b + "attn_v.weight", KV * Dh, E, s(E));
      w.q_norm = gen(b + "attn_q_norm.weight", Dh, 0.1f, 1.0f, seed);
      w.k_norm = gen(b + "attn_k_norm.weight", Dh, 0.1f, 1.0f, seed);
      w.wo = q8(b + "attn_output.weight", E, H * Dh, s(H * Dh));
      w.ffn_norm = gen(b + "ffn_norm.weight", E, 0.1f, 1.0f, seed);
      w.gate = q8(b + "ffn_gate.weight", F, E, s(E));
      w.up = q8(b + "ffn_up.weight", F, E, s(E));
      w.down = q8(b + "ffn_down.weight", E, F, s(F));
      layers.push_back(std::move(w));
    }
    out_norm = gen("output_norm.weight", E, 0.1f, 1.0f, seed);
    // RoPE table (qwen3.rope_table): iterative f32 theta, f64 cos/sin rounded to f32
    const int hd = Dh / 2;
    rcos.resize((size_t)n_ctx * hd);
    rsin.resize((size_t)n_ctx * hd);
    const float ts = std::pow(theta, -2.0f / (float)Dh);
    for (int p = 0; p < n_ctx; ++p) {
      float th = (float)p;
      for (int i = 0; i < hd; ++i) {
        rcos[(size_t)p * hd + i] = (float)std::cos((double)th);
        rsin[(size_t)p * hd + i] = (float)std::sin((double)th);
        th = th * ts;
      }
    }
    kc.assign((size_t)max_seqs * L * n_ctx * KV * Dh, 0);
    vc.assign((size_t)max_seqs * L * n_ctx * KV * Dh, 0);
  }

  // ggml rms_norm: sum of f32 squares in double, 1/sqrtf(mean + eps) in f32, then * w
  void rms_norm(const float* x, int n, const float* w, float* y) const {
    double ss = 0;
    for (int i = 0; i < n; ++i) ss += (double)(x[i] * x[i]);
    const float mean = (float)(ss / n);
    const float sc = 1.0f / std::sqrt(mean + eps);
    for (int i = 0; i < n; ++i) y[i] = (x[i] * sc) * w[i];
  }

  // y[N][O] = W . x rows (activations quantised per row)
  void matmul(const Q8& W, const float* x, int N, float* y, int64_t ldy) const {
    const int K = W.K, nb = K / 32;
    std::vector<int8_t> aq((size_t)N * K);
    std::vector<float> ad((size_t)N * nb);
#pragma omp parallel for schedule(static)
    for (int n = 0; n < N; ++n) quant_row_q8(x + (size_t)n * K, K, aq.data() + (size_t)n * K, ad.data() + (size_t)n * nb);
#pragma omp parallel for schedule(static)
    for (int o = 0; o < W.O; ++o) {
      const int8_t* wq = W.q.data() + (size_t)o * K;
      const float* wd = W.d.data() + (size_t)o * nb;
      for (int n = 0; n < N; ++n) y[(size_t)n * ldy + o] = dot_q8(wq, wd, aq.data() + (size_t)n * K, ad.data() + (size_t)n * nb, nb);
    }
  }

  void embed(const int32_t* ids, int n, int fp16_round, float* out) const {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < E; ++j) {
        const float v = tok.d[(size_t)ids[i] * (E / 32) + j / 32] * (float)tok.q[(size_t)ids[i] * E + j];
        out[(size_t)i * E + j] = fp16_round ? f16_round(v) : v;
      }
  }

  void rope(float* v, int pos) const {
    const int hd = Dh / 2;
    const float* c = rcos.data() + (size_t)pos * hd;
    const float* s = rsin.data() + (size_t)pos * hd;
    for (int i = 0; i < hd; ++i) {
      const float x0 = v[i], x1 = v[i + hd];
      v[i] = x0 * c[i] - x1 * s[i];
      v[i + hd] = x0 * s[i] + x1 * c[i];
    }
  }

  // x [N][E] at positions pos0.. of sequence `seq` -> logits [N or 1][V]
  void forward(int seq, const float* xin, int N, int pos0, int all_logits, float* logits) {
    std::vector<float> x(xin, xin + (size_t)N * E), h((size_t)N * E), q((size_t)N * H * Dh), k((size_t)N * KV * Dh),
        v((size_t)N * KV * Dh), o((size_t)N * H * Dh), g((size_t)N * F), u((size_t)N * F), y((size_t)N * E);
    const int T = pos0 + N, G = H / KV;
    const float scale = 1.0f / std::sqrt((float)Dh);
    for (int l = 0; l < L; ++l) {
      const LlmLayer& w = layers[l];
      uint16_t* K16 = kc.data() + ((size_t)seq * L + l) * n_ctx * KV * Dh;
      uint16_t* V16 = vc.data() + ((size_t)seq * L + l) * n_ctx * KV * Dh;
      for (int n = 0; n < N; ++n) rms_norm(x.data() + (size_t)n * E, E, w.attn_norm.data(), h.data() + (size_t)n * E);
      matmul(w.wq, h.data(), N, q.data(), H * Dh);
      matmul(w.wk, h.data(), N, k.data(), KV * Dh);
      matmul(w.wv, h.data(), N, v.data(), KV * Dh);
#pragma omp parallel for schedule(static)
      for (int n = 0; n < N; ++n) {
        std::vector<float> t(Dh);
        for (int hh = 0; hh < H; ++hh) {
          float* r = q.data() + ((size_t)n * H + hh) * Dh;
          rms_norm(r, Dh, w.q_norm.data(), t.data());
          std::copy(t.begin(), t.end(), r);
          rope(r, pos0 + n);
        }
        for (int hh = 0; hh < KV; ++hh) {
          float* r = k.data() + ((size_t)n * KV + hh) * Dh;
          rms_norm(r, Dh, w.k_norm.data(), t.data());
          std::copy(t.begin(), t.end(), r);
          rope(r, pos0 + n);
        }
        for (int i = 0; i < KV * Dh; ++i) {
          K16[(size_t)(pos0 + n) * KV * Dh + i] = f16_bits(k[(size_t)n * KV * Dh + i]);
          V16[(size_t)(pos0 + n) * KV * Dh + i] = f16_bits(v[(size_t)n * KV * Dh + i]);
        }
      }
      // causal attention over the f16 cache, f32 softmax
#pragma omp parallel for collapse(2) schedule(dynamic)
      for (int n = 0; n < N; ++n)
        for (int hh = 0; hh < H; ++hh) {
          const int pos = pos0 + n, kvh = hh / G;
          const float* qr = q.data() + ((size_t)n * H + hh) * Dh;
          std::vector<float> s(pos + 1), kf(Dh);
          float mx = -INFINITY;
          for (int j = 0; j <= pos; ++j) {
            const uint16_t* kr = K16 + (size_t)j * KV * Dh + kvh * Dh;
            float a = 0.f;
            for (int i = 0; i < Dh; ++i) a += qr[i] * f16_val(kr[i]);
            s[j] = a * scale;
            mx = std::max(mx, s[j]);
          }
          double z = 0;
          for (int j = 0; j <= pos; ++j) {
            s[j] = std::exp(s[j] - mx);
            z += s[j];
          }
          float* orow = o.data() + ((size_t)n * H + hh) * Dh;
          for (int i = 0; i < Dh; ++i) orow[i] = 0.f;
          for (int j = 0; j <= pos; ++j) {
            const float p = s[j] / (float)z;
            const uint16_t* vr = V16 + (size_t)j * KV * Dh + kvh * Dh;
            for (int i = 0; i < Dh; ++i) orow[i] += p * f16_val(vr[i]);
          }
        }
      (void)T;
      matmul(w.wo, o.data(), N, y.data(), E);
      for (size_t i = 0; i < x.size(); ++i) x[i] = x[i] + y[i];
      for (int n = 0; n < N; ++n) rms_norm(x.data() + (size_t)n * E, E, w.ffn_norm.data(), h.data() + (size_t)n * E);
      matmul(w.gate, h.data(), N, g.data(), F);
      matmul(w.up, h.data(), N, u.data(), F);
      for (size_t i = 0; i < g.size(); ++i) g[i] = (g[i] / (1.0f + std::exp(-g[i]))) * u[i];
      matmul(w.down, g.data(), N, y.data(), E);
      for (size_t i = 0; i < x.size(); ++i) x[i] = x[i] + y[i];
    }
    const int r0 = all_logits ? 0 : N - 1, nr = all_logits ? N : 1;
    std::vector<float> hn((size_t)nr * E);
    for (int n = 0; n < nr; ++n) rms_norm(x.data() + (size_t)(r0 + n) * E, E, out_norm.data(), hn.data() + (size_t)n * E);
    matmul(tok, hn.data(), nr, logits, V);
  }
};

}  // namespace

extern "C" {

int cref_threads(void) { return omp_get_max_threads(); }

void* cref_enc_create(const int32_t* cfg, uint32_t seed) {
  EncCfg c;
  std::memcpy(&c, cfg, sizeof(EncCfg));
  return new Encoder(c, seed);
}
void cref_enc_destroy(void* h) { delete (Encoder*)h; }
int cref_enc_forward(void* h, const float* audio, int64_t n_phys, int64_t valid, float* enc_out, float* ad_out,
                     int32_t* ids_out, float* margin_out, int32_t* tgt_out) {
  return ((Encoder*)h)->forward(audio, n_phys, valid, enc_out, ad_out, ids_out, margin_out, tgt_out);
}

void* cref_llm_create(const int32_t* cfg7, float rope_theta, float rms_eps, int32_t n_ctx, int32_t max_seqs,
                      uint32_t seed) {
  return new Llm(cfg7, rope_theta, rms_eps, n_ctx, max_seqs, seed);
}
void cref_llm_destroy(void* h) { delete (Llm*)h; }
void cref_llm_embed(void* h, const int32_t* ids, int32_t n, int32_t fp16_round, float* out) {
  ((Llm*)h)->embed(ids, n, fp16_round, out);
}
int cref_llm_forward(void* h, int32_t seq, const float* x, int32_t n, int32_t pos0, int32_t all_logits, float* logits) {
  Llm* m = (Llm*)h;
  if (seq < 0 || seq >= m->max_seqs || pos0 < 0 || pos0 + n > m->n_ctx) return -1;
  m->forward(seq, x, n, pos0, all_logits, logits);
  return 0;
}
// q8_0 blocks of a decoder tensor in ggml layout (fp16 d + 32 int8), for byte comparisons with the device copy
int cref_llm_tensor_q8(void* h, const char* name, uint8_t* out, int64_t n_bytes) {
  Llm* m = (Llm*)h;
  const Q8* t = nullptr;
  std::string nm(name);
  if (nm == "token_embd.weight") t = &m->tok;
  for (int l = 0; l < m->L && !t; ++l) {
    const std::string b = "blk." + std::to_string(l) + ".";
    const LlmLayer& w = m->layers[l];
    if (nm == b + "attn_q.weight") t = &w.wq;
    else if (nm == b + "attn_k.weight") t = &w.wk;
    else if (nm == b + "attn_v.weight") t = &w.wv;
    else if (nm == b + "attn_output.weight") t = &w.wo;
    else if (nm == b + "ffn_gate.weight") t = &w.gate;
    else if (nm == b + "ffn_up.weight") t = &w.up;
    else if (nm == b + "ffn_down.weight") t = &w.down;
  }
  if (!t || n_bytes != (int64_t)t->q.size() / 32 * 34) return -1;
  for (size_t b = 0; b < t->q.size() / 32; ++b) {
    const uint16_t d = f16_bits(t->d[b]);
    std::memcpy(out + b * 34, &d, 2);
    std::memcpy(out + b * 34 + 2, t->q.data() + b * 32, 32);
  }
  return 0;
}

}  // extern "C"
