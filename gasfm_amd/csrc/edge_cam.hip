// Edge prologue with the CAMERA-direction GATv2 attention fused in, and the camera attention's
// backward recomputing its source rows, gfx950.
//
// A block's edge prologue computes both convs' lin_l on P_hat = relu(LN(P)) (layers.py:232-234;
// PyG's lin_l) -- XL = [XLp | XLc], 32 + 32 features per edge -- and the camera direction's
// attention (Proj2View, layers.py:329-335) then reduces XLc over each camera's edges.  The edges
// are camera-major, so a camera segment is a contiguous run of the prologue's own 16-edge tiles:
//
//   edge_cam_fwd   over the camera plan's work items (one camera, <= max_piece edges each):
//                  XLp is written (in point-segment order through pos, as edge_prologue_fwd does)
//                  and XLc is consumed by an online softmax in registers -- never stored.
//   edge_cam_bwd   the camera attention's backward (gat_attn.hip attn_bwd_*): XLc recomputed from
//                  P (LayerNorm + 16 MFMAs per tile) instead of read back, dXLc written for
//                  gasfm_edge_prologue_bwd (which takes the two halves of dXL separately), dXR per
//                  camera, d att / d bias per workgroup.
// HBM per edge and block: the forward writes 256 B less (XLc) and the camera attention's forward
// read of XLc (128 B) is gone; the backward reads P (128 B) where it read XLc (128 B).
//
// MFMA orientation: the TRANSPOSED products XL^T = W P_hat^T (A = W from LDS, B = P_hat^T from the
// wave's LDS tile) leave lane (g = l >> 4, c = l & 15) holding features 16 ot + 4 g + r (r < 4) of
// EDGE c: one edge per lane column.  A head (8 features) is then 4 of the lane's registers plus
// the same 4 of lane l ^ 16, the per-edge softmax state is one per lane and head, and a lane's
// XLp / dXLc features are one float4 store per 16-feature tile (a row is 8 lanes x 16 B).
//
// Semantics are those of gasfm_gat_attn_fwd / _bwd on the camera plan: complete items write
// out[seg] (finalized with bias, or the raw acc), split items packed partial rows [acc 32 | max 4 |
// sum 4] for gasfm_gat_attn_combine; empty segments give out = bias, max = -inf, sum = 0; d bias
// sums gout over every segment (once, at its first item).
#include "edge_cam_common.hpp"

namespace gasfm {
namespace {

using namespace tile;

// =============================================================================================
// forward
// =============================================================================================
template <bool LN>
__global__ __launch_bounds__(kThreads, GASFM_CAM_MINW) void edge_cam_fwd_kernel(
    const float* __restrict__ P, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wpt, const float* __restrict__ bpt, const float* __restrict__ Wc,
    const float* __restrict__ bc, float* __restrict__ XLp, int64_t ldXLp, const int32_t* __restrict__ pos,
    const float* __restrict__ XR, int64_t ldXR, const float* __restrict__ att, const float* __restrict__ bias,
    float slope, const gasfm_work_item* __restrict__ items, int n_items, int finalize, float* __restrict__ out,
    int64_t ldOut, float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat,
    float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float Wl[kCamR ? NX * F : NX * LDA];  // slabs, or Wl[n][k] = [Wpt; Wc][n][k]
  __shared__ float tiles[kCamR ? 1 : kWaves][TR * LD34];
  if (kCamR) {
    stage_slabs32<NX, kThreads>([&](int q) { return q < F * F ? Wpt[q] : Wc[q - F * F]; }, Wl);
  } else {
    Stage<NX * F, kThreads> sw;
    sw.load([&](int q) { return q < F * F ? Wpt[q] : Wc[q - F * F]; });
    sw.store([&](int q, float v) { Wl[(q / F) * LDA + q % F] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T = tiles[kCamR ? 0 : wave];
  float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float g8[2][4], b8[2][4];  // gamma / beta at the slab features 16 u + 4 g + j
  if (LN) {
    g4 = *reinterpret_cast<const float4*>(gam + (lane & 7) * 4);
    b4 = *reinterpret_cast<const float4*>(bet + (lane & 7) * 4);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g8[u][j] = gam[16 * u + 4 * g + j];
        b8[u][j] = bet[16 * u + 4 * g + j];
      }
  }
  // this lane's features: point 16 ot + 4 g + r (ot = 0, 1); camera 16 q + 4 g + r (q = 0, 1),
  // head 2 q + (g >> 1)
  float bp[2][4], bcv[2][4], attv[2][4], biasv[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * q + 4 * g + r;
      bp[q][r] = bpt[f];
      bcv[q][r] = bc[f];
      attv[q][r] = att[f];
      biasv[q][r] = finalize ? bias[f] : 0.f;
    }
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;

  float4 np[2];
  f32x4 ns[2];
  int32_t npos = 0;  // point-order row of this lane's edge (column c)
  // branch-free: without pos the index load reads P's first words and is not used (a load under a
  // branch makes the join wait for every load in flight)
  const int32_t* posp = pos ? pos : reinterpret_cast<const int32_t*>(P);
  auto issue = [&](int64_t row0, int nrows) {
    if (kCamR)
      load_slabs32(P, row0, nrows, ns, lane);
    else
      load_rows(P, F, row0, nrows, np, lane);
    npos = posp[row0 + (c < nrows ? c : 0)];
  };
  auto rows_at = [](const gasfm_work_item& w, int64_t row0) { return int(w.end - row0 < TR ? w.end - row0 : TR); };

  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = items[gw];
    if (w.begin < w.end) issue(w.begin, rows_at(w, w.begin));
  }
  for (int it = gw; it < n_items; it += nw) {
    const int64_t seg = w.seg;
    float xr[2][4];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(XR + seg * ldXR + 16 * q + 4 * g);
      xr[q][0] = v.x, xr[q][1] = v.y, xr[q][2] = v.z, xr[q][3] = v.w;
    }
    float m[2] = {-INFINITY, -INFINITY}, s[2] = {0.f, 0.f};
    float a[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = items[it + nw];
    if (w.begin >= w.end && more && wn.begin < wn.end) issue(wn.begin, rows_at(wn, wn.begin));
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = rows_at(w, row0);
      f32x4 ph[2] = {ns[0], ns[1]};
      if (!kCamR) phat_to_lds<LN>(np, nrows, g4, b4, eps, T, lane);
      const int64_t dst = pos ? int64_t(npos) : row0 + (c < nrows ? c : 0);
      {  // the next tile (this item's, else the next item's first; the last one re-reads itself)
        int64_t r1 = row0;
        int n1 = nrows;
        if (row0 + TR < w.end) {
          r1 = row0 + TR;
          n1 = rows_at(w, r1);
        } else if (more && wn.begin < wn.end) {
          r1 = wn.begin;
          n1 = rows_at(wn, r1);
        }
        issue(r1, n1);
      }
      f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
      if (kCamR) {
        phat_slabs<LN>(ph, g8, b8, eps);
        xl_slabs<4>(reinterpret_cast<const float4*>(Wl), ph, acc, lane);
      } else {
        wave_sync();
        xl_t<4>(Wl, T, acc, c, g);
      }
      const bool valid = c < nrows;
      // point half: this lane's 2 x 4 features of edge c (non-temporal: streamed once by the point
      // attention)
      if (valid) {
        typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int ot = 0; ot < 2; ++ot)
          __builtin_nontemporal_store(v4f{acc[ot][0] + bp[ot][0], acc[ot][1] + bp[ot][1], acc[ot][2] + bp[ot][2],
                                          acc[ot][3] + bp[ot][3]},
                                      reinterpret_cast<v4f*>(XLp + dst * ldXLp + 16 * ot + 4 * g));
      }
      // camera half: logits of edge c, online softmax per head
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float xl[4], p = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xl[r] = acc[2 + q][r] + bcv[q][r];
          p = fmaf(leaky(xl[r] + xr[q][r], slope), attv[q][r], p);
        }
        p = xsum16(p);  // the head's other 4 features
        if (valid) {
          const float mn = fmaxf(m[q], p);
          const float sc = __expf(m[q] - mn), wt = __expf(p - mn);
          s[q] = fmaf(s[q], sc, wt);
#pragma unroll
          for (int r = 0; r < 4; ++r) a[q][r] = fmaf(a[q][r], sc, wt * xl[r]);
          m[q] = mn;
        }
      }
      if (!kCamR) wave_sync();  // T is rewritten by the next tile
    }
    // merge the 16 edge columns' states
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float M = row_max16(m[q]);
      const float f = (m[q] > -INFINITY) ? __expf(m[q] - M) : 0.f;
      const float S = group_sum<16>(s[q] * f);
      float A[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) A[r] = group_sum<16>(a[q][r] * f);
      if (c == 0) {
        const int f0 = 16 * q + 4 * g, h = 2 * q + (g >> 1);
        if (w.slot < 0) {
          const float inv = 1.f / (S + 1e-16f);
          float4 o;
          if (finalize)
            o = make_float4(fmaf(A[0], inv, biasv[q][0]), fmaf(A[1], inv, biasv[q][1]), fmaf(A[2], inv, biasv[q][2]),
                            fmaf(A[3], inv, biasv[q][3]));
          else
            o = make_float4(A[0], A[1], A[2], A[3]);
          *reinterpret_cast<float4*>(out + seg * ldOut + f0) = o;
          if ((g & 1) == 0) {
            seg_max[seg * ldStat + h] = M;
            seg_sum[seg * ldStat + h] = S;
          }
        } else {
          float* pr = part + int64_t(w.slot) * PART;
          *reinterpret_cast<float4*>(pr + f0) = make_float4(A[0], A[1], A[2], A[3]);
          if ((g & 1) == 0) {
            pr[F + h] = M;
            pr[F + H + h] = S;
          }
        }
      }
    }
    w = wn;
  }
}

// =============================================================================================
// backward of the camera attention, XLc recomputed from P
// =============================================================================================
// per workgroup partial row: [32 datt | 32 dbias]
constexpr int BP_PART = 2 * F;

template <bool LN>
__global__ __launch_bounds__(kThreads, GASFM_CAM_MINW) void edge_cam_bwd_kernel(
    const float* __restrict__ P, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wc, const float* __restrict__ bc, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, float slope, const float* __restrict__ out,
    int64_t ldOut, const float* __restrict__ seg_max, const float* __restrict__ seg_sum, int64_t ldStat,
    const float* __restrict__ gout, int64_t ldG, const gasfm_work_item* __restrict__ items, int n_items,
    float* __restrict__ dXLc, int64_t ldD, float* __restrict__ dXR, int64_t ldDXR, float* __restrict__ part_dxr,
    float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float Wl[kCamR ? F * F : F * LDA];  // slabs, or Wl[n][k] = Wc[n][k]
  __shared__ float tiles[kWaves][TR * LD34];  // (also the final reduction's scratch)
  if (kCamR) {
    stage_slabs32<F, kThreads>([&](int q) { return Wc[q]; }, Wl);
  } else {
    Stage<F * F, kThreads> sw;
    sw.load([&](int q) { return Wc[q]; });
    sw.store([&](int q, float v) { Wl[(q / F) * LDA + q % F] = v; });
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* T = tiles[wave];
  float4 g4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float g8[2][4], b8[2][4];  // gamma / beta at the slab features 16 u + 4 g + j
  if (LN) {
    g4 = *reinterpret_cast<const float4*>(gam + (lane & 7) * 4);
    b4 = *reinterpret_cast<const float4*>(bet + (lane & 7) * 4);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g8[u][j] = gam[16 * u + 4 * g + j];
        b8[u][j] = bet[16 * u + 4 * g + j];
      }
  }
  float bcv[2][4], attv[2][4], biasv[2][4], datt[2][4], dbias[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * q + 4 * g + r;
      bcv[q][r] = bc[f];
      attv[q][r] = att[f];
      biasv[q][r] = bias[f];
      datt[q][r] = dbias[q][r] = 0.f;
    }
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;

  float4 np[2];
  f32x4 ns[2];
  auto issue = [&](int64_t row0, int nrows) {
    if (kCamR)
      load_slabs32(P, row0, nrows, ns, lane);
    else
      load_rows(P, F, row0, nrows, np, lane);
  };
  auto rows_at = [](const gasfm_work_item& w, int64_t row0) { return int(w.end - row0 < TR ? w.end - row0 : TR); };
  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = items[gw];
    if (w.begin < w.end) issue(w.begin, rows_at(w, w.begin));
  }
  for (int it = gw; it < n_items; it += nw) {
    const int64_t seg = w.seg;
    // per-camera constants: XR, gout, out - bias at this lane's features; per head the forward's
    // max, 1 / (sum + 1e-16) and delta = sum_j alpha_j (g . XL_j) = g . (out - bias)
    float xr[2][4], gv[2][4], M[2], inv[2], delta[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int f0 = 16 * q + 4 * g, h = 2 * q + (g >> 1);
      const float4 x4 = *reinterpret_cast<const float4*>(XR + seg * ldXR + f0);
      const float4 g4v = *reinterpret_cast<const float4*>(gout + seg * ldG + f0);
      const float4 o4 = *reinterpret_cast<const float4*>(out + seg * ldOut + f0);
      xr[q][0] = x4.x, xr[q][1] = x4.y, xr[q][2] = x4.z, xr[q][3] = x4.w;
      gv[q][0] = g4v.x, gv[q][1] = g4v.y, gv[q][2] = g4v.z, gv[q][3] = g4v.w;
      const float o[4] = {o4.x, o4.y, o4.z, o4.w};
      float d = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) d = fmaf(gv[q][r], o[r] - biasv[q][r], d);
      delta[q] = xsum16(d);
      M[q] = seg_max[seg * ldStat + h];
      inv[q] = 1.f / (seg_sum[seg * ldStat + h] + 1e-16f);
    }
    const bool first = it == 0 || items[it - 1].seg != w.seg;
    if (first && c == 0) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) dbias[q][r] += gv[q][r];
    }
    float dxr[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = items[it + nw];
    if (w.begin >= w.end && more && wn.begin < wn.end) issue(wn.begin, rows_at(wn, wn.begin));
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = rows_at(w, row0);
      f32x4 ph[2] = {ns[0], ns[1]};
      if (!kCamR) phat_to_lds<LN>(np, nrows, g4, b4, eps, T, lane);
      {  // the next tile (see edge_cam_fwd_kernel)
        int64_t r1 = row0;
        int n1 = nrows;
        if (row0 + TR < w.end) {
          r1 = row0 + TR;
          n1 = rows_at(w, r1);
        } else if (more && wn.begin < wn.end) {
          r1 = wn.begin;
          n1 = rows_at(wn, r1);
        }
        issue(r1, n1);
      }
      f32x4 xc[2] = {zero4(), zero4()};
      if (kCamR) {
        phat_slabs<LN>(ph, g8, b8, eps);
        xl_slabs<2>(reinterpret_cast<const float4*>(Wl), ph, xc, lane);
      } else {
        wave_sync();
        xl_t<2>(Wl, T, xc, c, g);
      }
      const bool valid = c < nrows;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float xl[4], z[4], lz[4], p = 0.f, da = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xl[r] = xc[q][r] + bcv[q][r];
          z[r] = xl[r] + xr[q][r];
          lz[r] = leaky(z[r], slope);
          p = fmaf(lz[r], attv[q][r], p);
          da = fmaf(gv[q][r], xl[r], da);
        }
        p = xsum16(p);
        da = xsum16(da);
        const float alpha = valid ? __expf(p - M[q]) * inv[q] : 0.f;
        const float de = alpha * (da - delta[q]);
        float dx[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dz = de * attv[q][r] * (z[r] > 0.f ? 1.f : slope);
          dx[r] = fmaf(alpha, gv[q][r], dz);
          dxr[q][r] += dz;
          datt[q][r] = fmaf(de, lz[r], datt[q][r]);
        }
        if (valid)
          *reinterpret_cast<float4*>(dXLc + (row0 + c) * ldD + 16 * q + 4 * g) = make_float4(dx[0], dx[1], dx[2], dx[3]);
      }
      if (!kCamR) wave_sync();  // T is rewritten by the next tile
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = group_sum<16>(dxr[q][r]);
      if (c == 0) {
        float* d = (w.slot < 0) ? dXR + seg * ldDXR : part_dxr + int64_t(w.slot) * F;
        *reinterpret_cast<float4*>(d + 16 * q + 4 * g) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    w = wn;
  }
  // d att / d bias: sum over the 16 edge columns, then over the workgroup's waves (ordered)
  float v[16];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[q * 4 + r] = group_sum<16>(datt[q][r]);
      v[8 + q * 4 + r] = group_sum<16>(dbias[q][r]);
    }
  wg_reduce_ordered<16, kWaves, kWaves * TR * LD34>(v, &tiles[0][0], wave, lane);
  if (wave == 0 && c == 0) {
    float* o = part + int64_t(blockIdx.x) * BP_PART;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *reinterpret_cast<float4*>(o + 16 * q + 4 * g) = make_float4(v[q * 4], v[q * 4 + 1], v[q * 4 + 2], v[q * 4 + 3]);
      *reinterpret_cast<float4*>(o + F + 16 * q + 4 * g) =
          make_float4(v[8 + q * 4], v[8 + q * 4 + 1], v[8 + q * 4 + 2], v[8 + q * 4 + 3]);
    }
  }
}

// =============================================================================================
// backward, fused: camera attention + edge prologue of the block in ONE pass over the camera
// plan's items (gasfm_edge_cam_pbwd).  Per 16-edge tile, all in the T layout (lane (g, c): edge c,
// features 16 u + 4 g + j) except the weight-gradient operands:
//   P_hat = relu(LN(P)); XLc = Wc P_hat + bc recomputed; the camera attention's backward -> dXLc;
//   dP_hat = dXLp Wpt + dXLc Wc + dRes (scale Wp[:, :32])  (transposed products: B = T-layout rows);
//   dP = LN_bwd(mask * dP_hat) + dRes (stored), dgamma, dbeta;
//   dW += [dXLp | dXLc]^T P_hat, db  (C-layout operands through a per-wave LDS transpose).
// Replaces edge_cam_bwd + edge_prologue_bwd: dXLc (128 B per edge) is neither written nor read
// back, and P is read once.  Partial rows per workgroup: [dW 64x32 | db 64 | dgamma 32 | dbeta 32 |
// datt 32 | 0 (32: the bias gradient is the host's column sum of gout)].
// =============================================================================================
// Measured choices (tools/edge_bench.py, tools/gpu_ab_libs.sh): round 5's T-layout
// LayerNorm backward (below) replaced round 4's C-layout one (757 -> 675 us at config 4); dP is
// stored through a bounds-checked buffer descriptor per work item (rows past the item's end are
// dropped by the range check), so no per-row branch splits the tile's code; DWP's sums are LDS
// read-modify-writes.  Rejected in round 4: exec-mask-free tile loops, fewer registers held across
// tiles, dXLp in point order, block 0's epilogue folded in, XLc kept by the forward seam, static
// wave priority.
constexpr int PB2_PRO = NX * F + NX + 2 * F;  // the prologue_bwd part row
constexpr int PB2_PART = PB2_PRO + BP_PART;
constexpr int LDT = F + 4;                    // transpose tile row stride
constexpr int PB_NDW = 20;                    // (DWP) per-lane dWp sums: 16 MFMA values + 4 P0 terms

// The edge epilogues' backward folded into edge_cam_pbwd (round 3).  With SeamFn, the kernel that
// produces block b+1's dP is the one place where block b's epilogue gradient dP' (= that dP) is in
// registers in camera order, and block b's own edge_cam_pbwd later holds both dRes (= dP') and
// relu(LN_b(P_b)):
//   EPI (block b+1's launch): dSv_b[cam] = scale_e sum_e dP[e] (per camera item; split cameras as
//     partial rows), dP0_b[e] = scale_e We[:, 32:34]^T dP[e]
//   DWP (block b's launch): dWp_b = scale sum_e dRes[e]^T [relu(LN(P[e])) | P0[e]] as part rows
// which is everything edge_epilogue_bwd computed except dSp (segment_rowsum, point order).
struct PbwdEpi {
  const float* We;    // EPI: the previous block's lin_proj weight [32 x ldWe]
  int ldWe;
  float scale;        // EPI: the previous block's epilogue scale
  float* dSv;         // EPI: [m, 32]
  float* part_dsv;    // EPI: split-camera partial rows
  float* dP0;         // EPI: [E, 2] or null (no P0 skip input)
  const float* P0;    // DWP: [E, 2] or null
  int ldWpo;          // DWP: dWp row width in the part row (34 with P0, 32 without)
};

#ifndef GASFM_PBWD_MINW
#define GASFM_PBWD_MINW 2
#endif

// T-layout backward (round 5).  The LayerNorm backward runs where the forward's statistics are --
// lane (g, c) holds 8 features of edge c -- instead of in the C layout (4 edges x 2 features per
// lane): dP_hat comes out of the transposed products (A = the same weight slabs, B = the T-layout
// rows; acc[ot][r] = feature 16 ot + 4 g + r of edge c), so each row sum is 8 local adds and two
// cross-group swaps instead of a 16-lane DPP sum per edge, dP leaves as two 16-byte stores per lane,
// EPI's dP0 dot needs no transpose back and no statistics cross lanes.  The item's rows are read
// through bounds-checked buffer descriptors: rows past the item's end load as zeros, which zeroes
// every dead-edge quantity at its source (dXLp, dRes, P0; dXLc through alpha = 0), so no per-row
// masks remain.  Two transpose tiles per wave (was four): P_hat, dXLp and dXLc pass through tile A
// in turn (each read back at once), dRes and P0 sit in tile B for the dWp sums.  The attention bias
// gradient is not summed here: the host takes the column sum of gout over all targets
// (edge_block.replicated_dbias), which is also PyG's semantics for a target without edges.
// Why VALU: fp32 MFMA and VALU issue do not overlap on gfx950 (profiles/r5_mfma_valu_overlap.txt).
__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t rs, int off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
  return f32x4{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3])};
}
__device__ __forceinline__ void bstore4(const f32x4& x, __amdgpu_buffer_rsrc_t rs, int off) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
}
// descriptor over rows [begin, begin + len) of a row-major [*, ld] float tensor; its fields are
// wave-uniform and made provably so (a descriptor the compiler places in vector registers costs a
// waterfall loop around every load through it)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const float* X, int64_t ld, int begin, int len) {
  const uint64_t a = reinterpret_cast<uint64_t>(X + int64_t(begin) * ld);
  const uint64_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(a))));
  const uint64_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(a >> 32))));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(lo | (hi << 32)), 0,
                                           __builtin_amdgcn_readfirstlane(int(len * ld * 4)), 0x00020000);
}

template <bool LN, bool RES, bool EPI, bool DWP>
__global__ __launch_bounds__(kThreads, GASFM_PBWD_MINW) void edge_cam_pbwd_kernel(
    const float* __restrict__ P, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wpt, const float* __restrict__ Wc, const float* __restrict__ bc,
    const float* __restrict__ Wp, int ldWp, float scale, const float* __restrict__ XR, int64_t ldXR,
    const float* __restrict__ att, const float* __restrict__ bias, float slope, const float* __restrict__ out,
    int64_t ldOut, const float* __restrict__ seg_max, const float* __restrict__ seg_sum, int64_t ldStat,
    const float* __restrict__ gout, int64_t ldG, const gasfm_work_item* __restrict__ items, int n_items,
    const float* __restrict__ dXLp, int64_t ldXp, const float* __restrict__ dRes, float* __restrict__ dP,
    float* __restrict__ dXR, int64_t ldDXR, float* __restrict__ part_dxr, float* __restrict__ part, int64_t ldPart,
    PbwdEpi ep) {
  static_assert(!DWP || (LN && RES), "edge_cam_pbwd: the epilogue weight gradient needs relu(LN(P)) and dRes");
  // LDS: weight slabs (Wc for XLc; Wpt^T, Wc^T, (scale Wp)^T for dP_hat), the per-feature vectors,
  // per wave two 16 x 36 transpose tiles, per lane the running sums (DWP: dWp; EPI: dSv) at a lane
  // stride of an odd number of 16-byte quads (a 16-lane b128 access touches 16 distinct bank quads)
  constexpr int QW = F * F;  // floats per 32 x 32 slab set
  constexpr int OV = 4 * QW, OT = OV + (EPI ? 6 * F : 4 * F), WT = 2 * TR * LDT;
  constexpr int OD = OT + kWaves * WT;
  constexpr int NLS = DWP ? (PB_NDW + (EPI ? 8 : 0)) : (EPI ? 12 : 0);
  constexpr int NL = OD + kWaves * NLS * kW;
  __shared__ __attribute__((aligned(16))) float lds[NL];
  float* WcQ = lds;
  float* WptTQ = lds + QW;
  float* WcTQ = lds + 2 * QW;
  float* WqTQ = lds + 3 * QW;
  float* V = lds + OV;  // [gamma | beta | bc | att] (32 each), (EPI) [scale_e We[:, 32] | scale_e We[:, 33]]
  stage_slabs32<F, kThreads>([&](int q) { return Wc[q]; }, WcQ);
  stage_slabs32<F, kThreads>([&](int q) { return Wpt[(q % F) * F + q / F]; }, WptTQ);
  stage_slabs32<F, kThreads>([&](int q) { return Wc[(q % F) * F + q / F]; }, WcTQ);
  if (RES) stage_slabs32<F, kThreads>([&](int q) { return scale * Wp[(q % F) * ldWp + q / F]; }, WqTQ);
  if (threadIdx.x < F) {
    V[threadIdx.x] = LN ? gam[threadIdx.x] : 1.f;
    V[F + threadIdx.x] = LN ? bet[threadIdx.x] : 0.f;
    V[2 * F + threadIdx.x] = bc[threadIdx.x];
    V[3 * F + threadIdx.x] = att[threadIdx.x];
    if (EPI) {
      V[4 * F + threadIdx.x] = ep.dP0 ? ep.scale * ep.We[threadIdx.x * ep.ldWe + 32] : 0.f;
      V[5 * F + threadIdx.x] = ep.dP0 ? ep.scale * ep.We[threadIdx.x * ep.ldWe + 33] : 0.f;
    }
  }
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  float* Ta = lds + OT + wave * WT;  // P_hat, dXLp, dXLc in turn (each read back at once)
  float* Tb = Ta + TR * LDT;         // (DWP) dRes rows, P0 in columns 32, 33: read by the dWp sums
  float* Lw = lds + OD + (wave * kW + lane) * NLS;  // (DWP) this lane's dWp sums at Lw[0, 20)
  float* Ls = Lw + (DWP ? PB_NDW : 0);              // (EPI) the item's dSv column sums (T layout, 8)
#pragma unroll
  for (int k = 0; k < NLS; ++k) Lw[k] = 0.f;
  __syncthreads();
  // T-layout vector at this lane's features 16 q + 4 g .. + 3
  auto vecT = [&](int which, int q) {
    const float4 t = *reinterpret_cast<const float4*>(V + which * F + 16 * q + 4 * g);
    return f32x4{t.x, t.y, t.z, t.w};
  };
  // T -> C layout through tile T: writes the two slabs, returns the C-layout rows
  auto to_c = [&](float* T, const f32x4 (&t)[2], f32x4 (&o)[2]) {
    asm volatile("" ::: "memory");  // after the previous transpose's reads of the same tile
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<float4*>(T + c * LDT + 16 * u + 4 * g) = make_float4(t[u][0], t[u][1], t[u][2], t[u][3]);
    // one wave's LDS instructions execute in order: a compiler barrier suffices
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int ft = 0; ft < 2; ++ft)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[ft][r] = T[(4 * g + r) * LDT + 16 * ft + c];
  };
  f32x4 accW[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) accW[mt][0] = accW[mt][1] = zero4();
  float db[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 dg[2] = {zero4(), zero4()}, dbt[2] = {zero4(), zero4()}, datt[2] = {zero4(), zero4()};
  // the wave's first item (provably wave-uniform: the item loop, its branches and the descriptors
  // built from the items stay scalar -- no waterfall loops around the buffer loads)
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wave), nw = gridDim.x * kWaves;

  // next tile's rows of P, dXLp, dRes (T layout) and P0, one tile ahead; rows past the item's end
  // read as zeros (the descriptor's range check)
  f32x4 nPT[2], nXT[2], nRT[2];
  float2 nP0 = make_float2(0.f, 0.f);
  auto issue = [&](const gasfm_work_item& wi, int row0) {
    const int b = __builtin_amdgcn_readfirstlane(wi.begin), n = __builtin_amdgcn_readfirstlane(wi.end - wi.begin);
    const int r = row0 - b + c;  // edge c's row within the item
    const auto Prs = rows_rsrc(P, F, b, n);
    const auto Xrs = rows_rsrc(dXLp, ldXp, b, n);
#pragma unroll
    for (int u = 0; u < 2; ++u) nPT[u] = bload4(Prs, (r * F + 16 * u + 4 * g) * 4);
#pragma unroll
    for (int u = 0; u < 2; ++u) nXT[u] = bload4(Xrs, int((r * ldXp + 16 * u + 4 * g) * 4));
    if (RES) {
      const auto Rrs = rows_rsrc(dRes, F, b, n);
#pragma unroll
      for (int u = 0; u < 2; ++u) nRT[u] = bload4(Rrs, (r * F + 16 * u + 4 * g) * 4);
    }
    if (DWP && ep.P0) {  // (a global load: the compiler tail-merges a descriptor here into vector registers)
      const float2 t = *reinterpret_cast<const float2*>(ep.P0 + (int64_t(b) + (r < n ? r : 0)) * 2);
      nP0 = r < n ? t : make_float2(0.f, 0.f);
    }
  };
  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = uniform_item(items[gw]);
    if (w.begin < w.end) issue(w, w.begin);
  }
  for (int it = gw; it < n_items; it += nw) {
    const int64_t seg = w.seg;
    const int ibeg = w.begin, ilen = w.end - w.begin;
    const auto dPrs = rows_rsrc(dP, F, ibeg, ilen);
    // (EPI) dP0 rows of this item; without dP0 an empty range (every store dropped)
    const auto dP0rs = (EPI && ep.dP0) ? rows_rsrc(ep.dP0, 2, ibeg, ilen) : rows_rsrc(dP, F, ibeg, 0);
    // per-camera constants of the attention backward (edge_cam_bwd_kernel)
    f32x4 xr[2], gv[2];
    float M[2], inv[2], delta[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int f0 = 16 * q + 4 * g, h = 2 * q + (g >> 1);
      const float4 x4 = *reinterpret_cast<const float4*>(XR + seg * ldXR + f0);
      const float4 g4v = *reinterpret_cast<const float4*>(gout + seg * ldG + f0);
      const float4 o4 = *reinterpret_cast<const float4*>(out + seg * ldOut + f0);
      const float4 b4 = *reinterpret_cast<const float4*>(bias + f0);
      xr[q] = f32x4{x4.x, x4.y, x4.z, x4.w};
      gv[q] = f32x4{g4v.x, g4v.y, g4v.z, g4v.w};
      float d = fmaf(g4v.x, o4.x - b4.x, fmaf(g4v.y, o4.y - b4.y, fmaf(g4v.z, o4.z - b4.z, g4v.w * (o4.w - b4.w))));
      delta[q] = xsum16(d);
      M[q] = seg_max[seg * ldStat + h];
      inv[q] = 1.f / (seg_sum[seg * ldStat + h] + 1e-16f);
    }
    f32x4 dxr[2] = {zero4(), zero4()};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = uniform_item(items[it + nw]);
    if (w.begin >= w.end && more && wn.begin < wn.end) issue(wn, wn.begin);
    for (int row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = w.end - row0 < TR ? w.end - row0 : TR;
      f32x4 PT[2] = {nPT[0], nPT[1]}, XT[2] = {nXT[0], nXT[1]}, RT[2];
      if (RES) {
        RT[0] = nRT[0];
        RT[1] = nRT[1];
      }
      const float2 p0t = nP0;
      // the next tile: this item's, else the next item's first
      if (row0 + TR < w.end)
        issue(w, row0 + TR);
      else if (more && wn.begin < wn.end)
        issue(wn, wn.begin);
      const bool valid = c < nrows;
      // ---- LayerNorm of edge c (T layout): PT becomes xh, ph = relu(LN(P))
      f32x4 ph[2];
      float rstd = 1.f;
      if (LN) {  // packed math (ln_center / ln_affine, as the forward kernels)
        rstd = ln_center(PT, eps);
        float gs[2][4], bs[2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const f32x4 a = vecT(0, u), b = vecT(1, u);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            gs[u][j] = a[j];
            bs[u][j] = b[j];
          }
        }
        f32x4 xh[2];
        ln_affine(PT, rstd, gs, bs, ph, xh);
        PT[0] = xh[0];
        PT[1] = xh[1];
      } else {
        ph[0] = PT[0];
        ph[1] = PT[1];
      }
      // ---- C layout of P_hat (the weight gradients' B operand); dRes and P0 into tile B
      f32x4 phC[2];
      to_c(Ta, ph, phC);
      if (DWP) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
          *reinterpret_cast<float4*>(Tb + c * LDT + 16 * u + 4 * g) = make_float4(RT[u][0], RT[u][1], RT[u][2], RT[u][3]);
        if (g == 0) *reinterpret_cast<float2*>(Tb + c * LDT + 32) = p0t;
      }
      // ---- camera attention backward (T layout: edge c, features 16 q + 4 g + r)
      f32x4 xc[2] = {vecT(2, 0), vecT(2, 1)};  // b_c, then + Wc P_hat^T
      xl_slabs<2>(reinterpret_cast<const float4*>(WcQ), ph, xc, lane);
      f32x4 dXc[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 at = vecT(3, q);
        float z[4], lz[4], p = 0.f, da = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          z[r] = xc[q][r] + xr[q][r];
          lz[r] = leaky(z[r], slope);
          p = fmaf(lz[r], at[r], p);
          da = fmaf(gv[q][r], xc[q][r], da);
        }
        p = xsum16(p);
        da = xsum16(da);
        const float alpha = valid ? __expf(p - M[q]) * inv[q] : 0.f;
        const float de = alpha * (da - delta[q]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dz = de * at[r] * (z[r] > 0.f ? 1.f : slope);
          dXc[q][r] = fmaf(alpha, gv[q][r], dz);  // 0 for dead edges
          dxr[q][r] += dz;
          datt[q][r] = fmaf(de, lz[r], datt[q][r]);
        }
      }
      // ---- dP_hat (T layout) = dXLp Wpt + dXLc Wc (+ dRes scale Wp[:, :32])
      f32x4 dph[2] = {zero4(), zero4()};
      xl_slabs<2>(reinterpret_cast<const float4*>(WptTQ), XT, dph, lane);
      xl_slabs<2>(reinterpret_cast<const float4*>(WcTQ), dXc, dph, lane);
      if (RES) xl_slabs<2>(reinterpret_cast<const float4*>(WqTQ), RT, dph, lane);
      f32x4 XC[2], XcC[2];  // C layouts of dXLp, dXLc (the weight gradients' A operand)
      to_c(Ta, XT, XC);
      to_c(Ta, dXc, XcC);
      // ---- LayerNorm backward of edge c, dP (T layout)
      f32x4 dv[2];
      if (LN) {  // packed math: two features per v_pk_* instruction
        f32x2 gvv[2][2], s1p = {0.f, 0.f}, s2p = {0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const f32x4 a = vecT(0, u);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x2 dy = {ph[u][2 * h] > 0.f ? dph[u][2 * h] : 0.f,
                              ph[u][2 * h + 1] > 0.f ? dph[u][2 * h + 1] : 0.f};
            const f32x2 xh = pair(PT[u], h);
            set_pair(dg[u], h, __builtin_elementwise_fma(dy, xh, pair(dg[u], h)));
            set_pair(dbt[u], h, pair(dbt[u], h) + dy);
            const f32x2 gv = dy * pair(a, h);
            gvv[u][h] = gv;
            s1p += gv;
            s2p = __builtin_elementwise_fma(gv, xh, s2p);
          }
        }
        const float s1 = xsum32(xsum16(s1p.x + s1p.y)) * (1.f / F);
        const float s2 = xsum32(xsum16(s2p.x + s2p.y)) * (1.f / F);
        const f32x2 s1v = {s1, s1}, ms2 = {-s2, -s2}, r2 = {rstd, rstd};
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            // rstd ((gvv - s1) - xh s2) (+ dRes)
            const f32x2 t = __builtin_elementwise_fma(pair(PT[u], h), ms2, gvv[u][h] - s1v);
            set_pair(dv[u], h, RES ? __builtin_elementwise_fma(t, r2, pair(RT[u], h)) : t * r2);
          }
      } else {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) dv[u][j] = dph[u][j] + (RES ? RT[u][j] : 0.f);
      }
      // rows past the item's end fall outside the descriptor's range: the hardware drops them
#pragma unroll
      for (int u = 0; u < 2; ++u) bstore4(dv[u], dPrs, ((row0 - ibeg + c) * F + 16 * u + 4 * g) * 4);
      if (EPI) {
        // the previous block's epilogue: the item's column sums of dP (dSv; dead edges hold 0), and
        // dP0 = scale_e We[:, 32:34]^T dP per edge (a dot per lane, the 4 lane groups summed; group
        // 0 stores the pair, the other groups an out-of-range offset)
        float4* L4 = reinterpret_cast<float4*>(Ls);
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float4 t = L4[u];
          t.x += dv[u][0];
          t.y += dv[u][1];
          t.z += dv[u][2];
          t.w += dv[u][3];
          L4[u] = t;
          const f32x4 a = vecT(4, u), b = vecT(5, u);
          s0 = fmaf(dv[u][0], a[0], fmaf(dv[u][1], a[1], fmaf(dv[u][2], a[2], fmaf(dv[u][3], a[3], s0))));
          s1 = fmaf(dv[u][0], b[0], fmaf(dv[u][1], b[1], fmaf(dv[u][2], b[2], fmaf(dv[u][3], b[3], s1))));
        }
        s0 = sum_groups(s0);
        s1 = sum_groups(s1);
        const int off = g == 0 ? (row0 - ibeg + c) * 8 : 0x7ffffff0;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s0), dP0rs, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s1), dP0rs, off + 4, 0, 0);
      }
      // ---- dW += [dXLp | dXLc]^T relu(LN(P)), db (C layout, row 4 g + s at step s; dead rows 0)
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const float a = mt < 2 ? XC[mt][s2] : XcC[mt - 2][s2];
          db[mt] += a;
          accW[mt][0] = mfma16(a, phC[0][s2], accW[mt][0]);
          accW[mt][1] = mfma16(a, phC[1][s2], accW[mt][1]);
        }
      }
      if (DWP) {
        // this block's epilogue: dWp += dRes^T [relu(LN(P)) | P0] (dead rows are zeros), one
        // 16-feature half of dRes at a time, its rows and P0 read from tile B, the products added
        // into the lanes' LDS sums
#pragma unroll
        for (int ft = 0; ft < 2; ++ft) {
          float rr[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) rr[r] = Tb[(4 * g + r) * LDT + 16 * ft + c];
          f32x4 ap[2] = {zero4(), zero4()};
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) ap[nt] = mfma16(rr[s2], phC[nt][s2], ap[nt]);
          float a0[2] = {0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            a0[0] = fmaf(rr[r], Tb[(4 * g + r) * LDT + 32], a0[0]);
            a0[1] = fmaf(rr[r], Tb[(4 * g + r) * LDT + 33], a0[1]);
          }
          float* q = Lw + 10 * ft;
#pragma unroll
          for (int k = 0; k < 8; ++k) q[k] += ap[k / 4][k % 4];
          q[8] += a0[0];
          q[9] += a0[1];
        }
      }
      __builtin_amdgcn_wave_barrier();  // this tile's LDS reads before the next tile's writes
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = group_sum<16>(dxr[q][r]);
      if (c == 0) {
        float* d = (w.slot < 0) ? dXR + seg * ldDXR : part_dxr + int64_t(w.slot) * F;
        *reinterpret_cast<float4*>(d + 16 * q + 4 * g) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    if (EPI) {  // the item's dSv row: the 16 edge lanes of each group summed
      float4* L4 = reinterpret_cast<float4*>(Ls);
      float sv[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float4 t = L4[u];
        L4[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        sv[u][0] = group_sum<16>(t.x) * ep.scale;
        sv[u][1] = group_sum<16>(t.y) * ep.scale;
        sv[u][2] = group_sum<16>(t.z) * ep.scale;
        sv[u][3] = group_sum<16>(t.w) * ep.scale;
      }
      if (c == 0) {
        float* d = (w.slot < 0) ? ep.dSv + seg * F : ep.part_dsv + int64_t(w.slot) * F;
#pragma unroll
        for (int u = 0; u < 2; ++u)
          *reinterpret_cast<float4*>(d + 16 * u + 4 * g) = make_float4(sv[u][0], sv[u][1], sv[u][2], sv[u][3]);
      }
    }
    w = wn;
  }
  // workgroup reduction: 32 accW + 4 db (C layout) + 1 (dgamma / dbeta: the 16 edge lanes summed,
  // lane c keeps value c of its group) + 3 spare + 8 datt (edge lanes summed) + 8 spare (the bias
  // gradient is the host's) (+ DWP: the lanes' 20 dWp sums, read before the scratch is reused)
  constexpr int NV = 56 + (DWP ? PB_NDW : 0);
  float v[NV];
  if (DWP) {  // v[56 + (ft * 2 + nt) * 4 + r] = the MFMA sums, v[72 + ft * 2 + j] = the P0 terms
#pragma unroll
    for (int ft = 0; ft < 2; ++ft) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[56 + ft * 8 + k] = Lw[10 * ft + k];
#pragma unroll
      for (int j = 0; j < 2; ++j) v[72 + ft * 2 + j] = Lw[10 * ft + 8 + j];
    }
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[(mt * 2 + nt) * 4 + r] = accW[mt][nt][r];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) v[32 + mt] = db[mt];
  {
    float sel = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float t = group_sum<16>(k < 8 ? dg[k / 4][k % 4] : dbt[(k - 8) / 4][k % 4]);
      sel = c == k ? t : sel;
    }
    v[36] = sel;
  }
  v[37] = v[38] = v[39] = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[40 + q * 4 + r] = group_sum<16>(datt[q][r]);
      v[48 + q * 4 + r] = 0.f;
    }
  wg_reduce_ordered<NV, kWaves, NL>(v, lds, wave, lane);
  if (wave == 0) {
    float* o = part + int64_t(blockIdx.x) * ldPart;
    if (DWP) {  // [32 x ldWpo] after the prologue/attention part, scaled as the epilogue's
      float* od = o + PB2_PART;
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            od[(16 * ft + 4 * g + r) * ep.ldWpo + 16 * nt + c] = v[56 + (ft * 2 + nt) * 4 + r] * scale;
      float t0[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) t0[k] = sum_groups(v[72 + k]);
      if (ep.P0 && g == 0) {
#pragma unroll
        for (int ft = 0; ft < 2; ++ft)
#pragma unroll
          for (int j = 0; j < 2; ++j) od[(16 * ft + c) * ep.ldWpo + 32 + j] = t0[ft * 2 + j] * scale;
      }
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[(mt * 16 + 4 * g + r) * F + nt * 16 + c] = v[(mt * 2 + nt) * 4 + r];
    float tt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tt[k] = sum_groups(v[32 + k]);
    if (g == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) o[NX * F + mt * 16 + c] = tt[mt];
    }
    {  // dgamma / dbeta: lane (g, c) holds value c of group g: feature 16 (c / 4 % 2) + 4 g + c % 4
      const int k = c & 7;
      o[NX * F + NX + (c < 8 ? 0 : F) + 16 * (k >> 2) + 4 * g + (k & 3)] = v[36];
    }
    if (c == 0) {
      float* oa = o + PB2_PRO;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        *reinterpret_cast<float4*>(oa + 16 * q + 4 * g) =
            make_float4(v[40 + q * 4], v[40 + q * 4 + 1], v[40 + q * 4 + 2], v[40 + q * 4 + 3]);
        *reinterpret_cast<float4*>(oa + F + 16 * q + 4 * g) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
}

int grid_cam_pbwd(int n_items) {
  return resident_grid(reinterpret_cast<const void*>(&edge_cam_pbwd_kernel<true, true, false, false>), kThreads, 0,
                       n_items, kWaves);
}

int grid_cam_bwd(int n_items) {
  return resident_grid(reinterpret_cast<const void*>(&edge_cam_bwd_kernel<true>), kThreads, 0, n_items, kWaves);
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int32_t gasfm_edge_cam_bwd_part_rows(int32_t n_items) { return grid_cam_bwd(n_items > 0 ? n_items : 1); }
extern "C" int32_t gasfm_edge_cam_bwd_part_cols(void) { return BP_PART; }

extern "C" int gasfm_edge_cam_fwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                  const float* bpt, const float* Wc, const float* bc, float* XLp, int64_t ldXLp,
                                  const int32_t* pos, const float* XR, int64_t ldXR, const float* att,
                                  const float* bias, float slope, const gasfm_work_item* items, int32_t n_items,
                                  int32_t finalize, float* out, int64_t ldOut, float* seg_max, float* seg_sum,
                                  int64_t ldStat, float* part, void* stream) {
  GASFM_REQUIRE(n_items >= 0 && P && Wpt && bpt && Wc && bc && XLp && XR && att && items,
                "gasfm_edge_cam_fwd: null pointer");
  GASFM_REQUIRE((out && seg_max && seg_sum && (bias || !finalize)) || part, "gasfm_edge_cam_fwd: no outputs");
  GASFM_REQUIRE(ldXLp >= F && ldXLp % 4 == 0 && ldXR >= F && ldXR % 4 == 0 && (!out || (ldOut >= F && ldOut % 4 == 0)) &&
                    aligned16(P) && aligned16(XLp) && aligned16(XR) && (!out || aligned16(out)) &&
                    (!part || aligned16(part)) && (!ln_w || (aligned16(ln_w) && aligned16(ln_b))),
                "gasfm_edge_cam_fwd: 16-byte rows required");
  GASFM_REQUIRE(slope >= 0.f && slope <= 1.f, "gasfm_edge_cam_fwd: negative_slope %g outside [0, 1]", double(slope));
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  auto launch = [&](auto kern) {
    const int grid = resident_grid(reinterpret_cast<const void*>(kern), kThreads, 0, n_items, kWaves);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, P, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, ldXLp,
                       pos, XR, ldXR, att, bias, slope, items, n_items, finalize, out, ldOut, seg_max, seg_sum,
                       ldStat, part);
  };
  if (ln_w)
    launch(&edge_cam_fwd_kernel<true>);
  else
    launch(&edge_cam_fwd_kernel<false>);
  return launch_status("gasfm_edge_cam_fwd");
}

extern "C" int gasfm_edge_cam_bwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wc,
                                  const float* bc, const float* XR, int64_t ldXR, const float* att, const float* bias,
                                  float slope, const float* out, int64_t ldOut, const float* seg_max,
                                  const float* seg_sum, int64_t ldStat, const float* gout, int64_t ldG,
                                  const gasfm_work_item* items, int32_t n_items, float* dXLc, int64_t ldD, float* dXR,
                                  int64_t ldDXR, float* part_dxr, float* part, void* stream) {
  GASFM_REQUIRE(n_items >= 0 && P && Wc && bc && XR && att && bias && out && seg_max && seg_sum && gout && items &&
                    dXLc && dXR && part,
                "gasfm_edge_cam_bwd: null pointer");
  GASFM_REQUIRE(ldXR % 4 == 0 && ldOut % 4 == 0 && ldG % 4 == 0 && ldD % 4 == 0 && ldDXR % 4 == 0 && aligned16(P) &&
                    aligned16(XR) && aligned16(out) && aligned16(gout) && aligned16(dXLc) && aligned16(dXR) &&
                    (!part_dxr || aligned16(part_dxr)) && (!ln_w || (aligned16(ln_w) && aligned16(ln_b))),
                "gasfm_edge_cam_bwd: 16-byte rows required");
  GASFM_REQUIRE(slope >= 0.f && slope <= 1.f, "gasfm_edge_cam_bwd: negative_slope %g outside [0, 1]", double(slope));
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = grid_cam_bwd(n_items);
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, P, ln_w, ln_b, eps, Wc, bc, XR, ldXR, att, bias, slope,
                       out, ldOut, seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLc, ldD, dXR, ldDXR,
                       part_dxr, part);
  };
  if (ln_w)
    launch(&edge_cam_bwd_kernel<true>);
  else
    launch(&edge_cam_bwd_kernel<false>);
  return launch_status("gasfm_edge_cam_bwd");
}

extern "C" int32_t gasfm_edge_cam_pbwd_part_rows(int32_t n_items) { return grid_cam_pbwd(n_items > 0 ? n_items : 1); }
extern "C" int32_t gasfm_edge_cam_pbwd_part_cols(void) { return PB2_PART; }

extern "C" int gasfm_edge_cam_pbwd_ex(const float* P, const float* ln_w, const float* ln_b, float eps,
                                      const float* Wpt, const float* Wc, const float* bc, const float* Wp, int32_t ldWp,
                                      float scale, const float* XR, int64_t ldXR, const float* att, const float* bias,
                                      float slope, const float* out, int64_t ldOut, const float* seg_max,
                                      const float* seg_sum, int64_t ldStat, const float* gout, int64_t ldG,
                                      const gasfm_work_item* items, int32_t n_items, const float* dXLp, int64_t ldXp,
                                      const float* dRes, float* dP, float* dXR, int64_t ldDXR, float* part_dxr,
                                      float* part, int64_t ldPart, const float* We, int32_t ldWe, float scale_e,
                                      float* dSv_e, float* part_dsv_e, float* dP0_e, const float* P0, int32_t ldWpo,
                                      void* stream) {
  GASFM_REQUIRE(n_items >= 0 && P && Wpt && Wc && bc && XR && att && bias && out && seg_max && seg_sum && gout &&
                    items && dXLp && dP && dXR && part && (!dRes || (Wp && ldWp >= F)),
                "gasfm_edge_cam_pbwd: null pointer");
  GASFM_REQUIRE(ldXR % 4 == 0 && ldOut % 4 == 0 && ldG % 4 == 0 && ldXp % 4 == 0 && ldXp >= F && ldDXR % 4 == 0 &&
                    aligned16(P) && aligned16(XR) && aligned16(out) && aligned16(gout) && aligned16(dXLp) &&
                    aligned16(dP) && aligned16(dXR) && (!dRes || aligned16(dRes)) &&
                    (!part_dxr || aligned16(part_dxr)) && (!ln_w || (aligned16(ln_w) && aligned16(ln_b))),
                "gasfm_edge_cam_pbwd: 16-byte rows required");
  const bool epi = dSv_e != nullptr, dwp = ldWpo > 0;
  GASFM_REQUIRE(!epi || (We && ldWe >= F + (dP0_e ? 2 : 0) && (ln_w != nullptr) == (dRes != nullptr)),
                "gasfm_edge_cam_pbwd: the previous epilogue's outputs need its lin_proj weight (and LN == RES)");
  GASFM_REQUIRE(!dwp || (ln_w && dRes && ldWpo == (P0 ? F + 2 : F)),
                "gasfm_edge_cam_pbwd: the epilogue weight gradient needs LN, dRes and ldWpo = 32 (+2 with P0)");
  GASFM_REQUIRE(ldPart >= PB2_PART + (dwp ? int64_t(F) * ldWpo : 0), "gasfm_edge_cam_pbwd: part row too narrow");
  GASFM_REQUIRE(slope >= 0.f && slope <= 1.f, "gasfm_edge_cam_pbwd: negative_slope %g outside [0, 1]", double(slope));
  if (n_items == 0) return GASFM_OK;
  const PbwdEpi ep{We, ldWe, scale_e, dSv_e, part_dsv_e, dP0_e, P0, ldWpo};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = grid_cam_pbwd(n_items);
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, P, ln_w, ln_b, eps, Wpt, Wc, bc, Wp, ldWp, scale, XR,
                       ldXR, att, bias, slope, out, ldOut, seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLp,
                       ldXp, dRes, dP, dXR, ldDXR, part_dxr, part, ldPart, ep);
  };
  if (ln_w && dRes) {
    if (epi && dwp)
      launch(&edge_cam_pbwd_kernel<true, true, true, true>);
    else if (epi)
      launch(&edge_cam_pbwd_kernel<true, true, true, false>);
    else if (dwp)
      launch(&edge_cam_pbwd_kernel<true, true, false, true>);
    else
      launch(&edge_cam_pbwd_kernel<true, true, false, false>);
  } else if (ln_w) {
    launch(&edge_cam_pbwd_kernel<true, false, false, false>);
  } else if (dRes) {
    launch(&edge_cam_pbwd_kernel<false, true, false, false>);
  } else if (epi) {
    launch(&edge_cam_pbwd_kernel<false, false, true, false>);
  } else {
    launch(&edge_cam_pbwd_kernel<false, false, false, false>);
  }
  return launch_status("gasfm_edge_cam_pbwd");
}

extern "C" int gasfm_edge_cam_pbwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                   const float* Wc, const float* bc, const float* Wp, int32_t ldWp, float scale,
                                   const float* XR, int64_t ldXR, const float* att, const float* bias, float slope,
                                   const float* out, int64_t ldOut, const float* seg_max, const float* seg_sum,
                                   int64_t ldStat, const float* gout, int64_t ldG, const gasfm_work_item* items,
                                   int32_t n_items, const float* dXLp, int64_t ldXp, const float* dRes, float* dP,
                                   float* dXR, int64_t ldDXR, float* part_dxr, float* part, void* stream) {
  return gasfm_edge_cam_pbwd_ex(P, ln_w, ln_b, eps, Wpt, Wc, bc, Wp, ldWp, scale, XR, ldXR, att, bias, slope, out,
                                ldOut, seg_max, seg_sum, ldStat, gout, ldG, items, n_items, dXLp, ldXp, dRes, dP, dXR,
                                ldDXR, part_dxr, part, PB2_PART, nullptr, 0, 0.f, nullptr, nullptr, nullptr, nullptr, 0,
                                stream);
}
