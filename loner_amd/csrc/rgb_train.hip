// Colour-head training backward (camera phase), the kernel of lnr_rgb_train (rgb.hip launches it).
// Compiled on its own with -mllvm -amdgpu-mfma-vgpr-form (loner_amd/build.py FILE_FLAGS): the MFMA results land
// in VGPRs, where the VALU consumes every one of them (round 5: 394 -> 51 v_accvgpr moves per tile).
#include "rgb.hpp"

namespace lnr {

// ------------------------------------------------------------------ colour-head training backward, v2
// The same contract as k_rgb_bwd_tiles (the forward re-run bit-identically to the render; the chain
// dO -> dH_NH -> ... -> dH_0 -> d_enc on fp16 MFMA operands at per-wave power-of-two scales; fp32 weight
// gradients reduced in a fixed order), laid out for the VALU and LDS budget that bound round 4's kernel
// (profiles/r05_pmc_CAM.txt: 194 K VALU instructions per wave against 12.5 K MFMA, 60 % of the LDS cycles bank
// conflicts of 2-byte staging, one wave per SIMD waiting 40 % of its time):
//  * activations stay packed fp16 (v_cvt_pk_f16_f32 + v_pk_max_f16: the ReLU of the rounded value, which is
//    the rounding of the ReLU), and the ReLU masks are AND masks taken from those halves;
//  * each layer's input X_l and scaled gradient dY_l go to LDS as [sample][neuron] rows of 8-byte chunks
//    (one ds_write_b64 per 4 neurons of a sample, XOR-swizzled by row pair), and the weight-gradient MFMAs
//    read them back transposed with ds_read_b64_tr_b16 (neuron on the lane, 4 samples per lane: the
//    16x16x16 operand), conflict-free;
//  * 8 waves (two per SIMD: the serial per-tile chain of one wave hides behind the other's) take a 16-sample
//    tile each per iteration; wave w owns rows 16 (w/2) .. +15 of every weight matrix, half of its column tiles,
//    each at its own running power-of-two scale; two barriers per 128 samples (images complete, images read);
//  * W_l lives in one LDS image, read by rows for the forward and transposed for the backward (W_l^T);
//  * the output layer's gradient (3 x 64) is each wave's own: its tile's H_NH and scaled dO go through the
//    wave's own rows of the dY images (before its backward writes them) into 16x16x16 MFMAs at a running scale.
// Scales: a layer's scale comes from the wave's largest |gradient| before the ReLU mask (k_rgb_bwd_tiles:
// after), so it is at most one power of two finer than it could be; deterministic either way.
typedef uint32_t u32x4v_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v_t __attribute__((ext_vector_type(2)));
constexpr int kBw2Waves = kRgbBwd2Waves;
constexpr int kBw2Cols = 16 * kBw2Waves;  // samples per workgroup iteration

// Rows of 16 8-byte chunks (64 halves): chunk ch of row r at dword 32 r + 2 (ch ^ f(r)).  The swizzles are chosen
// per image for every access the kernel makes to it, by the banking rules of MI355X_MICROARCH.md's LDS table (stores:
// (a/4) mod 32 in 16-lane groups for b64, 8-lane groups for b128; b64 and transposed reads: mod 64 in 32-lane
// halves; b128 reads: mod 64 in four 16-lane groups); an image read or written 16 bytes at a time keeps f even, so
// a chunk pair stays adjacent and in order:
//  * the per-tile images X_l, dY_l ([sample][neuron], 8-byte accesses only): f = bits (r2, r1, r3, r0) of r as chunk
//    bits 3..0.  A store instruction's 16 rows (one chunk each) meet 16 distinct positions, a transposed read's
//    rows 16 s + 4 g + q (g = 0, 1 or 2, 3) x 4 chunks and a b64 row read's 16 rows x 2 chunks 64 distinct banks;
//  * the weight images W_0, W_l: f = 4 ((r >> 1) mod 4), conflict-free for the forward's 16-byte row reads and
//    W_0's transposed reads; W_l's (wperm-ordered) transposed reads keep a 2-way conflict on half their groups,
//    which no single-bit-per-position swizzle with an even f removes.
// The first layout (that f for every image) spent 42 % of the LDS cycles on bank conflicts (profiles/r05_pmc_CAM.txt),
// mostly the 4-way conflicting stores of the per-tile images.  (tools/lds_banks_rgb.py counts every access.)
__device__ __forceinline__ uint32_t swt(uint32_t r, uint32_t ch) {
  const uint32_t f = (((r >> 1) & 3u) << 2) | (((r >> 3) & 1u) << 1) | (r & 1u);
  return 32u * r + 2u * (ch ^ f);
}
__device__ __forceinline__ uint32_t sww(uint32_t r, uint32_t ch) { return 32u * r + 2u * (ch ^ (((r >> 1) & 3u) << 2)); }
// W_l images: logical in-chunk lc = in / 4 = 8s + 4h + g stored at chunk 8s + 2g + h, so the forward's
// hid_perm(s, g, .) operand is one 16-byte row read; the transposed read's 4 consecutive in-indices stay one chunk
__device__ __forceinline__ uint32_t wperm(uint32_t lc) { return 8u * (lc >> 3) + 2u * (lc & 3u) + ((lc >> 2) & 1u); }
// [sample][32 halves] rows of 8 chunks (X_0): f = 2 ((r >> 1) mod 4), conflict-free for the 16-byte stores and the
// transposed reads
__device__ __forceinline__ uint32_t sw32(uint32_t r, uint32_t ch) { return 16u * r + 2u * (ch ^ (((r >> 1) & 3u) << 1)); }

template <int NH>
struct Bw2Buf {
  uint32_t x0[kBw2Cols * 16];                 // X_0's 32 colour-grid features, [sample][32 halves]
  _Float16 sh[kBw2Waves][16];                 // X_0's 16 SH features, one set per tile (one ray)
  uint32_t h[NH > 0 ? NH : 1][kBw2Cols * 32];  // X_1 .. X_NH = H_0 .. H_{NH-1}
  uint32_t dy[NH + 1][kBw2Cols * 32];         // dH_0 .. dH_NH at the source wave's scale
  float inv[kBw2Waves][NH + 1];               // 1 / that scale
  int valid[kBw2Waves];
};
template <int NH>
struct Bw2Lds {
  uint32_t w0[64 * 32];                       // W_0 [hid][48 in + 16 zeros], rows by 16 B for the forward, transposed for d_enc
  uint32_t wt[NH > 0 ? NH : 1][64 * 32];      // W_1 .. W_NH [out][in]: rows (in hid_perm order) and transposed
  half8_t ao[2][64];                          // the output layer's A operands per lane: W_out (rows by channel)
  half8_t aot[4][64];                         //   and W_out^T (k = channel), conflict-free 16-byte reads
  Bw2Buf<NH> buf;
};
// (after the loop) the output layer's gradient per wave, over the dY images
typedef float Bw2Red[kBw2Waves][3][64];

__device__ __forceinline__ void lds_st64(uint32_t* p, uint32_t x, uint32_t y) {
  *reinterpret_cast<u32x2v_t*>(__builtin_assume_aligned(p, 8)) = u32x2v_t{x, y};
}
__device__ __forceinline__ uint32_t pk_scaled(float x, float y, float s) {
  half2v_t h = {(_Float16)(x * s), (_Float16)(y * s)};
  return __builtin_bit_cast(uint32_t, h);
}
__device__ __forceinline__ half8_t pk_operand(const uint32_t (&v)[8], int s) {
  const u32x4v_t u = {v[4 * s], v[4 * s + 1], v[4 * s + 2], v[4 * s + 3]};
  return __builtin_bit_cast(half8_t, u);
}
template <int CTRL>
__device__ __forceinline__ float row_dpp(float v) {  // row_shr by CTRL's shift; lanes shifted in read 0
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float max_abs16(const float4_t (&acc)[4]) {
  float m = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) m = fmaxf(m, fmaxf(fmaxf(fabsf(acc[t][0]), fabsf(acc[t][1])), fmaxf(fabsf(acc[t][2]), fabsf(acc[t][3]))));
  return m;
}

// Owner step of one matrix: acc tiles (row tile wid / 2, column tiles ct0 + m, m < CT) += dY X^T over the valid
// source tiles, at the running scale `run`.  XI: the X image (nullptr: X_0, whose column tiles 0, 1 come from x0
// and 2 from the tiles' SH values).
template <int NH, int CT>
__device__ __forceinline__ void bw2_owner(const Bw2Buf<NH>& B, int l, const uint32_t* xi, float4_t (&acc)[2],
                                          float& run, int ct0) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int tq = (lane >> 2) & 3, tp = lane & 3;
  const uint32_t rt = (uint32_t)wid >> 1;
  int vd[kBw2Waves];
  float iv[kBw2Waves];
  float imax = 0.f;
#pragma unroll
  for (int sw = 0; sw < kBw2Waves; ++sw) {  // wave-uniform: through the scalar unit
    vd[sw] = __builtin_amdgcn_readfirstlane(B.valid[sw]);
    iv[sw] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(B.inv[sw][l])));
    if (vd[sw]) imax = fmaxf(imax, iv[sw]);
  }
  if (imax == 0.f) return;
  const float s_new = __builtin_amdgcn_rcpf(imax);  // exact: a power of two
  if (s_new < run) {  // wave-uniform
    if (run != INFINITY) {
      const float f = s_new / run;
#pragma unroll
      for (int m = 0; m < CT; ++m) acc[m] *= f;
    }
    run = s_new;
  }
#pragma unroll
  for (int sw = 0; sw < kBw2Waves; ++sw) {
    if (!vd[sw]) continue;
    const uint32_t r = 16u * sw + 4u * g + tq;  // the transposed read's row (sample) for this lane
    const _Float16 f = (_Float16)(run * iv[sw]);  // run / s_sw = 2^-k, k >= 0
    const half4_t fv = {f, f, f, f};
    const half4_t ya = lds_tr16(&B.dy[l][swt(r, 4u * rt + tp)]) * fv;
#pragma unroll
    for (int m = 0; m < CT; ++m) {
      const uint32_t ct = (uint32_t)ct0 + m;
      half4_t xb;
      if (xi != nullptr) {
        xb = lds_tr16(&xi[swt(r, 4u * ct + tp)]);
      } else if (ct < 2) {
        xb = lds_tr16(&B.x0[sw32(r, 4u * ct + tp)]);
      } else {
        const _Float16 v = B.sh[sw][c];
        xb = half4_t{v, v, v, v};
      }
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x16f16(ya, xb, acc[m], 0, 0, 0);
    }
  }
}

template <int NH>
__global__ void __launch_bounds__(64 * kBw2Waves) k_rgb_bwd2(RgbArgs a, float* __restrict__ d_enc,
                                                              float* __restrict__ slab) {
  __shared__ Bw2Lds<NH> sm;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int tq = (lane >> 2) & 3, tp = lane & 3;
  // ---- weights: W_0, W_l and the output layer's operands in LDS
  const uint16_t* wo = a.w + rgb_layer_offset<NH>(NH + 1);  // (16, 64): rows 0..2 are the colour channels
  if (wid == 0) {
    const int ch = c & 3;  // every 4-row group of the output tile holds the three channels (row 4g + q = channel q)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const half8_t z = {};
      sm.ao[s2][lane] = ch < 3 ? ld_half8_perm(wo + ch * kRgbWidth, s2, g) : z;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      half8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j)  // A = Wout^T: [hid 16t + c][k = output 8g + j], outputs 0..2 only
        v[j] = (g == 0 && j < 3) ? __builtin_bit_cast(_Float16, wo[j * kRgbWidth + 16 * t + c]) : (_Float16)0.f;
      sm.aot[t][lane] = v;
    }
  }
  for (int i = threadIdx.x; i < NH * 64 * 16; i += 64 * kBw2Waves) {  // W_l images, 8-byte chunks
    const int l = i >> 10, r = (i >> 4) & 63, ch = i & 15;
    const uint16_t* src = a.w + rgb_layer_offset<NH>(l + 1) + r * kRgbWidth + 4 * ch;
    lds_st64(&sm.wt[l][sww(r, wperm(ch))], (uint32_t)src[0] | ((uint32_t)src[1] << 16), (uint32_t)src[2] | ((uint32_t)src[3] << 16));
  }
  for (int i = threadIdx.x; i < 64 * 16; i += 64 * kBw2Waves) {  // W_0 image, natural order, zero columns 48..63
    const int r = i >> 4, ch = i & 15;
    const uint16_t* src = a.w + r * kRgbIn + 4 * ch;
    lds_st64(&sm.w0[sww(r, ch)], ch < 12 ? (uint32_t)src[0] | ((uint32_t)src[1] << 16) : 0u,
             ch < 12 ? (uint32_t)src[2] | ((uint32_t)src[3] << 16) : 0u);
  }
  // ---- weight-gradient accumulators: rows 16 (wid / 2) .. of W_0 (column tiles 0, 1 or 2) and of each W_l
  // (column tiles 2 (wid & 1) + m)
  float4_t acc0[2], acch[NH > 0 ? NH : 1][2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    acc0[m] = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int l = 0; l < NH; ++l) acch[l][m] = float4_t{0.f, 0.f, 0.f, 0.f};
  }
  float run0 = INFINITY, runh[NH > 0 ? NH : 1];
#pragma unroll
  for (int l = 0; l < NH; ++l) runh[l] = INFINITY;
  float4_t acco[4];  // output layer: d W_out[channel 4g + q][16m + c] of this wave's tiles (rows 0..2 real)
#pragma unroll
  for (int m = 0; m < 4; ++m) acco[m] = float4_t{0.f, 0.f, 0.f, 0.f};
  float runo = INFINITY;
  __syncthreads();

  // the live tiles only (k_rgb_render flagged them and zeroed the others' d_enc; k_rgb_tile_list listed them)
  const int64_t n_tiles = (int64_t)a.tile_count[0];
  const int64_t per_iter = (int64_t)gridDim.x * kBw2Waves;
  const int64_t n_iter = (n_tiles + per_iter - 1) / per_iter;
  float2* denc = reinterpret_cast<float2*>(d_enc);
  float lmax[4] = {0.f, 0.f, 0.f, 0.f};  // max |d_enc| of this lane's levels 2g, 2g + 1, 8 + 2g, 9 + 2g
  uint32_t nx[4];
  float nw = 0.f, ng[3] = {0.f, 0.f, 0.f}, nd[3] = {0.f, 0.f, 0.f};
  const uint32_t tpr = (uint32_t)(a.S / 16);
  int64_t pf_pos = (int64_t)blockIdx.x * kBw2Waves + wid, pf_tile = 0;
  auto prefetch = [&]() {
    if (pf_pos < n_tiles) {
      pf_tile = a.tile_list[pf_pos];
      const int64_t m0 = pf_tile * 16, ray = (int64_t)((uint32_t)pf_tile / tpr);
#pragma unroll
      for (int q = 0; q < 4; ++q) nx[q] = a.enc[(int64_t)(4 * g + q) * a.enc_stride + m0 + c];
      nw = a.weights[m0 + c];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        ng[k] = a.g[3 * ray + k];
        nd[k] = a.rays[13 * ray + 6 + k];
      }
    }
    pf_pos += per_iter;
  };
  prefetch();
  for (int64_t it = 0; it < n_iter; ++it) {
    Bw2Buf<NH>& B = sm.buf;
    const int64_t pos = it * per_iter + (int64_t)blockIdx.x * kBw2Waves + wid;
    const bool valid = pos < n_tiles;
    const int64_t tile = pf_tile;  // (the prefetch below moves pf_tile on)
    bool skip = true;
    if (valid) {
      uint32_t ex[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) ex[q] = nx[q];
      const float w_s = nw;
      float g_r[3], sh[16];
#pragma unroll
      for (int k = 0; k < 3; ++k) g_r[k] = ng[k];
      sh_eval<4>((nd[0] + 1.0f) / 2.0f, (nd[1] + 1.0f) / 2.0f, (nd[2] + 1.0f) / 2.0f, sh);
      prefetch();
      skip = __ballot(w_s != 0.f) == 0ull;  // all 16 weights exactly 0: no gradient anywhere in the tile
      const int64_t n0 = tile * 16;
      if (skip) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int lvl = 8 * m + 2 * g;
          denc[(int64_t)lvl * a.enc_stride + n0 + c] = make_float2(0.f, 0.f);
          denc[(int64_t)(lvl + 1) * a.enc_stride + n0 + c] = make_float2(0.f, 0.f);
        }
      } else {
        const uint32_t row = 16u * wid + c;
        // X_0: the encodings (already fp16 pairs) and the tile's SH values
        *reinterpret_cast<u32x4v_t*>(__builtin_assume_aligned(&B.x0[sw32(row, 2u * g)], 16)) = u32x4v_t{ex[0], ex[1], ex[2], ex[3]};
        const half8_t benc = __builtin_bit_cast(half8_t, u32x4v_t{ex[0], ex[1], ex[2], ex[3]});
        // (sh[8 g + j] by a bit select: a lane-dependent index into a register array would go to scratch)
        half8_t bsh;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t lo = __float_as_uint(sh[j]), hi = __float_as_uint(sh[8 + j]);
          bsh[j] = g < 2 ? (_Float16)__uint_as_float(g ? hi : lo) : (_Float16)0.f;
        }
        if (c == 0 && g < 2) *reinterpret_cast<half8_t*>(&B.sh[wid][8 * g]) = bsh;
        // forward (as k_rgb_render): H_l packed (hp: the current layer), staged as X_{l+1} for l < NH; H_NH goes to
        // this wave's rows of dy[NH] (the output layer's gradient reads it there, and the backward its mask)
        uint32_t hp[8];
        {
          float4_t ac[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {  // W_0[16t + c][8g + j] and [32 + 8g + j] (SH; zero columns for g >= 2)
            const uint32_t r0 = 16u * t + c;
            const half8_t a0 = __builtin_bit_cast(half8_t, *reinterpret_cast<const u32x4v_t*>(__builtin_assume_aligned(&sm.w0[sww(r0, 2u * g)], 16)));
            const half8_t as = __builtin_bit_cast(half8_t, *reinterpret_cast<const u32x4v_t*>(__builtin_assume_aligned(&sm.w0[sww(r0, 8u + 2u * g)], 16)));
            ac[t] = float4_t{0.f, 0.f, 0.f, 0.f};
            ac[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, benc, ac[t], 0, 0, 0);
            ac[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as, bsh, ac[t], 0, 0, 0);
            hp[2 * t] = pk_relu(ac[t][0], ac[t][1]);
            hp[2 * t + 1] = pk_relu(ac[t][2], ac[t][3]);
          }
        }
#pragma unroll
        for (int l = 0; l < NH; ++l) {
#pragma unroll
          for (int t = 0; t < 4; ++t) lds_st64(&B.h[l][swt(row, 4u * t + g)], hp[2 * t], hp[2 * t + 1]);
          const half8_t b0 = pk_operand(hp, 0), b1 = pk_operand(hp, 1);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            half8_t w[2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)  // W_{l+1}[out 16t + c][k = in hid_perm(s2, g, j)]: one 16-byte row read
              w[s2] = __builtin_bit_cast(half8_t, *reinterpret_cast<const u32x4v_t*>(
                                                      __builtin_assume_aligned(&sm.wt[l][sww(16u * t + c, 8u * s2 + 2u * g)], 16)));
            float4_t ac = {0.f, 0.f, 0.f, 0.f};
            ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[0], b0, ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[1], b1, ac, 0, 0, 0);
            hp[2 * t] = pk_relu(ac[0], ac[1]);
            hp[2 * t + 1] = pk_relu(ac[2], ac[3]);
          }
        }
        float4_t o = {0.f, 0.f, 0.f, 0.f};
        o = __builtin_amdgcn_mfma_f32_16x16x32_f16(sm.ao[0][lane], pk_operand(hp, 0), o, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_16x16x32_f16(sm.ao[1][lane], pk_operand(hp, 1), o, 0, 0, 0);
        // dL/dlogit of sample c, in every lane (rows 4g .. 4g+2 of the output tile are the channels)
        float dl[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float hc = round_f16(o[k]);
          const float cl = round_f16(1.0f / (1.0f + expf(-hc)));
          dl[k] = g_r[k] * w_s * cl * (1.0f - cl);
        }
        float scale = grad_scale(wave_max_nonneg(fmaxf(fabsf(dl[0]), fmaxf(fabsf(dl[1]), fabsf(dl[2])))));
        {  // the output layer's weight gradient dW_out += dO H_NH^T on MFMA (K = this tile's samples): H_NH and the
           // scaled dO are staged in this wave's own rows of dy[NH] and dy[0], which its backward overwrites below
          uint32_t* hs = B.dy[NH];
#pragma unroll
          for (int t = 0; t < 4; ++t) lds_st64(&hs[swt(row, 4u * t + g)], hp[2 * t], hp[2 * t + 1]);
          // [3 channels][16 samples] in this wave's rows of dy[0] (of the otherwise unused h image when NH = 0,
          // where dy[0] is dy[NH])
          _Float16* ds = reinterpret_cast<_Float16*>(NH > 0 ? &B.dy[0][512u * wid] : &B.h[0][512u * wid]);
          if (g == 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) ds[16 * k + c] = (_Float16)(dl[k] * scale);
          }
          if (scale < runo) {  // wave-uniform
            if (runo != INFINITY) {
              const float f = scale / runo;
#pragma unroll
              for (int m = 0; m < 4; ++m) acco[m] *= f;
            }
            runo = scale;
          }
          const _Float16 f = (_Float16)(runo * __builtin_amdgcn_rcpf(scale));  // 2^-k, k >= 0
          const half4_t fv = {f, f, f, f};
          const u32x2v_t dv = *reinterpret_cast<const u32x2v_t*>(__builtin_assume_aligned(&ds[16 * (c < 3 ? c : 0) + 4 * g], 8));
          const half4_t ya = c < 3 ? __builtin_bit_cast(half4_t, dv) * fv : half4_t{0, 0, 0, 0};
          const uint32_t rr = 16u * wid + 4u * g + tq;
#pragma unroll
          for (int m = 0; m < 4; ++m)
            acco[m] = __builtin_amdgcn_mfma_f32_16x16x16f16(ya, lds_tr16(&hs[swt(rr, 4u * m + tp)]), acco[m], 0, 0, 0);
        }
        half8_t bo = {};
#pragma unroll
        for (int k = 0; k < 3; ++k) bo[k] = g == 0 ? (_Float16)(dl[k] * scale) : (_Float16)0.f;
        float4_t ac[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          ac[t] = float4_t{0.f, 0.f, 0.f, 0.f};
          ac[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(sm.aot[t][lane], bo, ac[t], 0, 0, 0);
        }
        // dH_NH .. dH_0: rescale, mask, stage, propagate
        uint32_t dp[8];
#pragma unroll
        for (int l = NH; l >= 0; --l) {
          const float k2 = grad_scale(wave_max_nonneg(max_abs16(ac)));
          scale *= k2;
          const uint32_t* hl = l == NH ? B.dy[NH] : B.h[l < NH ? l : 0];  // H_l, this wave's rows (the mask)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const u32x2v_t hv = *reinterpret_cast<const u32x2v_t*>(__builtin_assume_aligned(&hl[swt(row, 4u * t + g)], 8));
            dp[2 * t] = pk_scaled(ac[t][0], ac[t][1], k2) & pk_nonzero_mask(hv.x);
            dp[2 * t + 1] = pk_scaled(ac[t][2], ac[t][3], k2) & pk_nonzero_mask(hv.y);
            lds_st64(&B.dy[l][swt(row, 4u * t + g)], dp[2 * t], dp[2 * t + 1]);
          }
          if (lane == 0) B.inv[wid][l] = __builtin_amdgcn_rcpf(scale);  // exact: scale is a power of two
          if (l == 0) break;
          const half8_t b0 = pk_operand(dp, 0), b1 = pk_operand(dp, 1);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            half8_t w[2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {  // W_l^T [in 16t + i][k = out hid_perm(s2, g, j)]
              const half4_t lo = lds_tr16(&sm.wt[l - 1][sww(32u * s2 + 4u * g + tq, wperm(4u * t + tp))]);
              const half4_t hi = lds_tr16(&sm.wt[l - 1][sww(32u * s2 + 16u + 4u * g + tq, wperm(4u * t + tp))]);
              w[s2] = half8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
            ac[t] = float4_t{0.f, 0.f, 0.f, 0.f};
            ac[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[0], b0, ac[t], 0, 0, 0);
            ac[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[1], b1, ac[t], 0, 0, 0);
          }
        }
        // d_enc = W0[:, :32]^T dH_0 (true value: / scale)
        const half8_t b0 = pk_operand(dp, 0), b1 = pk_operand(dp, 1);
        const float inv = __builtin_amdgcn_rcpf(scale);  // exact: a power of two
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          half8_t w[2];
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {  // W_0^T [in 16m + i][k = hid hid_perm(s2, g, j)]
            const half4_t lo = lds_tr16(&sm.w0[sww(32u * s2 + 4u * g + tq, 4u * m + tp)]);
            const half4_t hi = lds_tr16(&sm.w0[sww(32u * s2 + 16u + 4u * g + tq, 4u * m + tp)]);
            w[s2] = half8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
          float4_t e = {0.f, 0.f, 0.f, 0.f};
          e = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[0], b0, e, 0, 0, 0);
          e = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[1], b1, e, 0, 0, 0);
          const int lvl = 8 * m + 2 * g;
          const float2 q0 = make_float2(e[0] * inv, e[1] * inv), q1 = make_float2(e[2] * inv, e[3] * inv);
          denc[(int64_t)lvl * a.enc_stride + n0 + c] = q0;
          denc[(int64_t)(lvl + 1) * a.enc_stride + n0 + c] = q1;
          lmax[2 * m] = fmaxf(lmax[2 * m], fmaxf(fabsf(q0.x), fabsf(q0.y)));
          lmax[2 * m + 1] = fmaxf(lmax[2 * m + 1], fmaxf(fabsf(q1.x), fabsf(q1.y)));
        }
      }
    }
    if (lane == 0) B.valid[wid] = (valid && !skip) ? 1 : 0;
    lds_barrier();  // the images complete
    // owners: rows 16 (wid / 2) .. of dW_l += dY_l X_l^T over the 8 source tiles
    if ((wid & 1) == 0)
      bw2_owner<NH, 2>(B, 0, nullptr, acc0, run0, 0);
    else
      bw2_owner<NH, 1>(B, 0, nullptr, acc0, run0, 2);
#pragma unroll
    for (int l = 0; l < NH; ++l) bw2_owner<NH, 2>(B, l + 1, B.h[l], acch[l], runh[l], 2 * (wid & 1));
    lds_barrier();  // the images read: the next iteration may write them
  }
  // ---- weight gradients to this workgroup's slab
  float* sb = slab + (int64_t)blockIdx.x * rgb_mlp_params<NH>();
  const int rt = wid >> 1;
  {
    const float inv = run0 == INFINITY ? 0.f : 1.0f / run0;
    const int ct0 = (wid & 1) ? 2 : 0, nct = (wid & 1) ? 1 : 2;
#pragma unroll
    for (int m = 0; m < 2; ++m)
      if (m < nct) {
#pragma unroll
        for (int q = 0; q < 4; ++q) sb[(16 * rt + 4 * g + q) * kRgbIn + 16 * (ct0 + m) + c] = acc0[m][q] * inv;
      }
  }
#pragma unroll
  for (int l = 0; l < NH; ++l) {
    float* mat = sb + rgb_layer_offset<NH>(l + 1);
    const float inv = runh[l] == INFINITY ? 0.f : 1.0f / runh[l];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) mat[(16 * rt + 4 * g + q) * kRgbWidth + 16 * (2 * (wid & 1) + m) + c] = acch[l][m][q] * inv;
  }
  // the output layer: rows 0..2 of each wave's tiles, summed over the waves in a fixed order (in the dY images:
  // every wave passed the loop's last barrier, after the last reads of them)
  Bw2Red& red = *reinterpret_cast<Bw2Red*>(&sm.buf.dy[0][0]);
  if (g == 0) {
    const float inv = runo == INFINITY ? 0.f : 1.0f / runo;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int q = 0; q < 3; ++q) red[wid][q][16 * m + c] = acco[m][q] * inv;
  }
  __syncthreads();
  {
    float* mo = sb + rgb_layer_offset<NH>(NH + 1);
    for (int i = threadIdx.x; i < kRgbOutPad * kRgbWidth; i += 64 * kBw2Waves) {
      const int k = i / kRgbWidth, n = i % kRgbWidth;
      float v = 0.f;
      if (k < 3) {
#pragma unroll
        for (int w = 0; w < kBw2Waves; ++w) v += red[w][k][n];
      }
      mo[i] = v;
    }
  }
  if (a.denc_max) {  // the colour grid backward's record scales: 16-lane row max, one atomicMax per wave and level
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = lmax[q];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
      if (c == 0 && v > 0.f)
        atomicMax(reinterpret_cast<uint32_t*>(a.denc_max) + (q >> 1) * 8 + 2 * g + (q & 1), __float_as_uint(v));
    }
  }
}


}  // namespace lnr

void lnr::launch_rgb_bwd2(int NH, const RgbArgs& a, float* d_enc, float* slab, int nb, hipStream_t st) {
  switch (NH) {
    case 0: hipLaunchKernelGGL(k_rgb_bwd2<0>, dim3(nb), dim3(64 * kBw2Waves), 0, st, a, d_enc, slab); break;
    case 1: hipLaunchKernelGGL(k_rgb_bwd2<1>, dim3(nb), dim3(64 * kBw2Waves), 0, st, a, d_enc, slab); break;
    case 2: hipLaunchKernelGGL(k_rgb_bwd2<2>, dim3(nb), dim3(64 * kBw2Waves), 0, st, a, d_enc, slab); break;
    default: hipLaunchKernelGGL(k_rgb_bwd2<3>, dim3(nb), dim3(64 * kBw2Waves), 0, st, a, d_enc, slab); break;
  }
}
