// hipcc-flags: -mllvm --amdgpu-sched-strategy=max-ilp
// The forward seam (gasfm_edge_seam_fwd, gasfm_edge0_seam_fwd), split out of edge_cam.hip (round 6) so
// that it compiles under the ILP-maximising machine scheduler: 485 -> 467 us per config-4 launch
// (tools/edge_bench.py, profiles/r6_ab_sched.txt) while edge_cam_pbwd stays on the default
// scheduler (677 -> 692 us under max-ilp).  build.py reads the first line's hipcc flags.
#include "edge_cam_common.hpp"

namespace gasfm {
namespace {

using namespace tile;

// =============================================================================================
// forward seam: block b's edge epilogue + block b+1's prologue and camera attention in one pass
// (gasfm_edge_seam_fwd).  Per 16-edge tile of the camera plan's items (edge c on lane column c):
//   P_hat_b = relu(LN_b(P_b)),  Y = Wp_b[:, :32] P_hat_b^T                      (T layout, MFMA)
//   P' = P_b + scale (Y + bp + Sg + Wp_b[:, 32:34] P0 + Sp[pt] + Sv[cam])       stored
//   then exactly edge_cam_fwd on P' (LN_{b+1}, XL, point half stored, camera softmax).
// Replaces edge_epilogue_fwd + edge_cam_fwd: P' is never read back (128 B per edge), and the
// camera of a camera item is fixed, so Sv[cam] is one row per item.  Per-feature vectors live in
// LDS (read as float4 at the lane's features 16 q + 4 g .. + 3).
// =============================================================================================
struct SeamEpi {
  const float* P;     // P_b [E, 32]
  const float* P0;    // [E, 2] or null
  const int32_t* pt;  // point of each edge
  const float* gam;   // LN_b
  const float* bet;
  float eps;
  const float* Wp;    // [32 x ldWp]
  int ldWp;
  const float* bp;
  const float* Sp;    // [n, 32]
  const float* Sv;    // [m, ldSv]
  int64_t ldSv;
  const float* Sg;    // [32]
  float scale;
  float* Pout;        // P' [E, 32]
  // block 0's epilogue (EP0): P [E, 2], gam / bet = LN_a, Wp [32 x 2], and
  const float* gb;    // LN_b [2]
  const float* bb;
  const float* Wsk;   // skip projection [32 x 2]
  const float* bsk;   // [32]
};

#ifndef GASFM_SEAM_MINW
#define GASFM_SEAM_MINW 2
#endif
// The seam's memory order (round 3, tools/gpu_seam_ab.sh): the Sp[pt] rows of the next tile are
// gathered half a tile ahead (issued after this tile's P' store, from the next tile's point indices,
// which are the first of the next tile's requests), and the P' / XL stores are unconditional (a lane
// past the item's end rewrites its clamped row with that row's own values), so no store sits under a
// branch and the compiler's vmcnt bookkeeping stays exact (a store under a branch makes every later
// wait assume the store-free path, i.e. wait for younger loads too).  Measured and rejected: no
// branches at all (duplicate stores, select-based softmax update), the gather at the tile's own
// start, LDS-staged rows two tiles ahead, XCD-contiguous item dealing, static wave priority, XLc kept
// for the backward.
// EP0: block 0's epilogue (edge0_epilogue_fwd, 2-wide P) as the seam's first half:
//   P' = Wsk relu(LN_b(P)) + bsk + scale (Wp relu(LN_a(P)) + bp + Sg + Sp[pt] + Sv[cam])
// computed per lane on its 8 features (2-wide products: no MFMA), in edge0_epilogue_fwd's order.
template <bool LN, bool EP0>
__global__ __launch_bounds__(kThreads, GASFM_SEAM_MINW) void edge_seam_fwd_kernel(
    SeamEpi ep, const float* __restrict__ gam, const float* __restrict__ bet, float eps,
    const float* __restrict__ Wpt, const float* __restrict__ bpt, const float* __restrict__ Wc,
    const float* __restrict__ bc, float* __restrict__ XLp, int64_t ldXLp, const int32_t* __restrict__ pos,
    const float* __restrict__ XR, int64_t ldXR, const float* __restrict__ att, const float* __restrict__ bias,
    float slope, const gasfm_work_item* __restrict__ items, int n_items, int finalize, float* __restrict__ out,
    int64_t ldOut, float* __restrict__ seg_max, float* __restrict__ seg_sum, int64_t ldStat,
    float* __restrict__ part) {
  // vector table (32 floats each): 0 gamma_b 1 beta_b 2 bp+Sg 3 Wp[:,32] 4 Wp[:,33] 5 gamma 6 beta
  // 7 bpt 8 bc 9 att 10 bias; EP0: 0 Wsk[:,0] 1 Wsk[:,1] 2 bp+Sg 3 Wp[:,0] 4 Wp[:,1] 11 bsk
  __shared__ __attribute__((aligned(16))) float Wl[NX * F];   // [Wpt; Wc] slabs
  __shared__ __attribute__((aligned(16))) float WpQ[EP0 ? 4 : F * F];  // Wp_b[:, :32] slabs
  __shared__ __attribute__((aligned(16))) float V[12 * F];
  stage_slabs32<NX, kThreads>([&](int q) { return q < F * F ? Wpt[q] : Wc[q - F * F]; }, Wl);
  if (!EP0) stage_slabs32<F, kThreads>([&](int q) { return ep.Wp[(q / F) * ep.ldWp + q % F]; }, WpQ);
  if (threadIdx.x < F) {
    const int f = threadIdx.x;
    V[f] = EP0 ? ep.Wsk[2 * f] : ep.gam[f];
    V[F + f] = EP0 ? ep.Wsk[2 * f + 1] : ep.bet[f];
    V[2 * F + f] = ep.bp[f] + ep.Sg[f];
    V[3 * F + f] = EP0 ? ep.Wp[2 * f] : (ep.P0 ? ep.Wp[f * ep.ldWp + 32] : 0.f);
    V[4 * F + f] = EP0 ? ep.Wp[2 * f + 1] : (ep.P0 ? ep.Wp[f * ep.ldWp + 33] : 0.f);
    V[11 * F + f] = EP0 ? ep.bsk[f] : 0.f;
    V[5 * F + f] = LN ? gam[f] : 1.f;
    V[6 * F + f] = LN ? bet[f] : 0.f;
    V[7 * F + f] = bpt[f];
    V[8 * F + f] = bc[f];
    V[9 * F + f] = att[f];
    V[10 * F + f] = finalize ? bias[f] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & (kW - 1), wave = threadIdx.x / kW;
  const int c = lane & 15, g = lane >> 4;
  // (EP0) LN_a and LN_b over the 2 input features
  const float ga0 = EP0 ? ep.gam[0] : 0.f, ga1 = EP0 ? ep.gam[1] : 0.f, ba0 = EP0 ? ep.bet[0] : 0.f,
              ba1 = EP0 ? ep.bet[1] : 0.f, gb0 = EP0 ? ep.gb[0] : 0.f, gb1 = EP0 ? ep.gb[1] : 0.f,
              bb0 = EP0 ? ep.bb[0] : 0.f, bb1 = EP0 ? ep.bb[1] : 0.f;
  auto vec = [&](int which, int q) {
    const float4 t = *reinterpret_cast<const float4*>(V + which * F + 16 * q + 4 * g);
    return f32x4{t.x, t.y, t.z, t.w};
  };
  const int gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;
  // next tile: P_b slabs, the edge's point and P0 pair, its point-order row (all branch-free)
  f32x4 ns[2];
  int32_t npos = 0, npt = 0;
  float2 nq = make_float2(0.f, 0.f);
  const int32_t* posp = pos ? pos : reinterpret_cast<const int32_t*>(ep.P);
  const float* p0p = EP0 ? ep.P : (ep.P0 ? ep.P0 : ep.P);  // EP0: the 2-wide P row itself
  f32x4 nsp[2];  // Sp[pt] of the next tile
  auto issue = [&](int64_t row0, int nrows) {
    const int64_t e = row0 + (c < nrows ? c : 0);
    npt = ep.pt[e];  // first: waiting for it does not wait for the P rows
    if (!EP0) load_slabs32(ep.P, row0, nrows, ns, lane);
    npos = posp[e];
    nq = *reinterpret_cast<const float2*>(p0p + e * 2);
  };
  auto issue_sp = [&]() {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float4 t = *reinterpret_cast<const float4*>(ep.Sp + int64_t(npt) * F + 16 * q + 4 * g);
      nsp[q] = f32x4{t.x, t.y, t.z, t.w};
    }
  };
  // an item's first tile outside the tile loop: the Sp rows before the P rows, so that (as on the
  // loop's own path, where the tile's stores follow them) younger requests follow the Sp rows when
  // the loop is entered -- the compiler's wait counts are the minimum over the entering paths
  auto issue_first = [&](int64_t row0, int nrows) {
    npt = ep.pt[row0 + (c < nrows ? c : 0)];
    issue_sp();
    issue(row0, nrows);
  };
  auto rows_at = [](const gasfm_work_item& w, int64_t row0) { return int(w.end - row0 < TR ? w.end - row0 : TR); };

  gasfm_work_item w{0, 0, 0, -1};
  if (gw < n_items) {
    w = items[gw];
    if (w.begin < w.end) {
      issue_first(w.begin, rows_at(w, w.begin));
    }
  }
  for (int it = gw; it < n_items; it += nw) {
    const int64_t seg = w.seg;
    f32x4 xr[2], sv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(XR + seg * ldXR + 16 * q + 4 * g);
      xr[q] = f32x4{v.x, v.y, v.z, v.w};
      const float4 t = *reinterpret_cast<const float4*>(ep.Sv + seg * ep.ldSv + 16 * q + 4 * g);
      sv[q] = f32x4{t.x, t.y, t.z, t.w};
    }
    float m[2] = {-INFINITY, -INFINITY}, s[2] = {0.f, 0.f};
    f32x4 a[2] = {zero4(), zero4()};
    gasfm_work_item wn{0, 0, 0, -1};
    const bool more = it + nw < n_items;
    if (more) wn = items[it + nw];
    if (w.begin >= w.end && more && wn.begin < wn.end) {
      issue_first(wn.begin, rows_at(wn, wn.begin));
    }
    for (int64_t row0 = w.begin; row0 < w.end; row0 += TR) {
      const int nrows = rows_at(w, row0);
      f32x4 pb[2] = {ns[0], ns[1]};
      f32x4 sp[2] = {nsp[0], nsp[1]};
      // lanes past the item's end hold row0's values (clamped loads) and store them to row0's own
      // row: with pos == nullptr, row0 + c would belong to the next item (another wave's rows)
      const int64_t dst = pos ? int64_t(npos) : row0 + (c < nrows ? c : 0);
      const float2 q0 = nq;
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
      const bool valid = c < nrows;
      // ---- epilogue of block b (T layout)
      f32x4 pn[2];  // P' (this block's output, the next block's input)
      if (EP0) {
        // block 0: 2-wide P (q0), LN_a / LN_b over its 2 features (edge0_epilogue_fwd's order)
        const float mean = 0.5f * (q0.x + q0.y);
        const float d0 = q0.x - mean, d1 = q0.y - mean;
        const float rs = rsq_normal(0.5f * (d0 * d0 + d1 * d1) + ep.eps);
        const float xh0 = d0 * rs, xh1 = d1 * rs;
        const float ha0 = fmaxf(fmaf(xh0, ga0, ba0), 0.f), ha1 = fmaxf(fmaf(xh1, ga1, ba1), 0.f);
        const float hb0 = fmaxf(fmaf(xh0, gb0, bb0), 0.f), hb1 = fmaxf(fmaf(xh1, gb1, bb1), 0.f);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 ka = vec(0, q), kb = vec(1, q), cs = vec(2, q), wa = vec(3, q), wb = vec(4, q), bs = vec(11, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = fmaf(wa[r], ha0, fmaf(wb[r], ha1, cs[r])) + sp[q][r] + sv[q][r];
            pn[q][r] = fmaf(d, ep.scale, fmaf(ka[r], hb0, fmaf(kb[r], hb1, bs[r])));
          }
        }
      } else {
        f32x4 ph[2] = {pb[0], pb[1]};
        {
          float gs[2][4], bs[2][4];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const f32x4 ga = vec(0, q), be = vec(1, q);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              gs[q][r] = ga[r];
              bs[q][r] = be[r];
            }
          }
          phat_slabs<true>(ph, gs, bs, ep.eps);
        }
        f32x4 y[2] = {zero4(), zero4()};
        xl_slabs<2>(reinterpret_cast<const float4*>(WpQ), ph, y, lane);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 cs = vec(2, q), w32 = vec(3, q), w33 = vec(4, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float d = y[q][r] + cs[r];
            d = fmaf(w32[r], q0.x, fmaf(w33[r], q0.y, d));
            // (d + Sv) + Sp: the gathered Sp row is consumed last (not hoisted to the tile's top)
            d = (d + sv[q][r]) + sp[q][r];
            pn[q][r] = fmaf(d, ep.scale, pb[q][r]);
          }
        }
      }
      // not hoisted towards the point-index load it waits for: the address is formed from npt only
      // once P' exists
      asm volatile("" : "+v"(npt) : "v"(pn[0][0]), "v"(pn[1][3]));
      issue_sp();
      {
        const int64_t prow = row0 + (valid ? c : 0);
#pragma unroll
        for (int q = 0; q < 2; ++q)
          *reinterpret_cast<float4*>(ep.Pout + prow * F + 16 * q + 4 * g) =
              make_float4(pn[q][0], pn[q][1], pn[q][2], pn[q][3]);
      }
      // ---- prologue + camera attention of block b+1 on P' (edge_cam_fwd_kernel)
      {
        float gs[2][4], bs[2][4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f32x4 ga = vec(5, q), be = vec(6, q);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gs[q][r] = ga[r];
            bs[q][r] = be[r];
          }
        }
        phat_slabs<LN>(pn, gs, bs, eps);
      }
      f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
      xl_slabs<4>(reinterpret_cast<const float4*>(Wl), pn, acc, lane);
      {
        typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
          const f32x4 b = vec(7, ot);
          __builtin_nontemporal_store(v4f{acc[ot][0] + b[0], acc[ot][1] + b[1], acc[ot][2] + b[2], acc[ot][3] + b[3]},
                                      reinterpret_cast<v4f*>(XLp + dst * ldXLp + 16 * ot + 4 * g));
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 bcq = vec(8, q), atq = vec(9, q);
        float xl[4], p = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xl[r] = acc[2 + q][r] + bcq[r];
          p = fmaf(leaky(xl[r] + xr[q][r], slope), atq[r], p);
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
    }
    // merge the 16 edge columns' states (edge_cam_fwd_kernel)
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
          if (finalize) {
            const f32x4 bq = vec(10, q);
            o = make_float4(fmaf(A[0], inv, bq[0]), fmaf(A[1], inv, bq[1]), fmaf(A[2], inv, bq[2]),
                            fmaf(A[3], inv, bq[3]));
          } else {
            o = make_float4(A[0], A[1], A[2], A[3]);
          }
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

}  // namespace
}  // namespace gasfm

using namespace gasfm;

extern "C" int gasfm_edge_seam_fwd(const float* Pb, const float* P0, const int32_t* pt, const float* ln_wb,
                                   const float* ln_bb, float eps_b, const float* Wp, int32_t ldWp, const float* bp,
                                   const float* Sp, const float* Sv, int64_t ldSv, const float* Sg, float scale,
                                   float* Pout, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                   const float* bpt, const float* Wc, const float* bc, float* XLp, int64_t ldXLp,
                                   const int32_t* pos, const float* XR, int64_t ldXR, const float* att,
                                   const float* bias, float slope, const gasfm_work_item* items, int32_t n_items,
                                   int32_t finalize, float* out, int64_t ldOut, float* seg_max, float* seg_sum,
                                   int64_t ldStat, float* part, void* stream) {
  GASFM_REQUIRE(n_items >= 0 && Pb && pt && ln_wb && ln_bb && Wp && bp && Sp && Sv && Sg && Pout && Wpt && bpt &&
                    Wc && bc && XLp && XR && att && items,
                "gasfm_edge_seam_fwd: null pointer");
  GASFM_REQUIRE(ldWp >= (P0 ? F + 2 : F), "gasfm_edge_seam_fwd: ldWp");
  GASFM_REQUIRE((out && seg_max && seg_sum && (bias || !finalize)) || part, "gasfm_edge_seam_fwd: no outputs");
  GASFM_REQUIRE(ldXLp >= F && ldXLp % 4 == 0 && ldXR >= F && ldXR % 4 == 0 && ldSv >= F && ldSv % 4 == 0 &&
                    (!out || (ldOut >= F && ldOut % 4 == 0)) && aligned16(Pb) && aligned16(Pout) && aligned16(Sp) &&
                    aligned16(Sv) && aligned16(XLp) && aligned16(XR) && (!out || aligned16(out)) &&
                    (!part || aligned16(part)) && (!P0 || (reinterpret_cast<uintptr_t>(P0) % 8 == 0)),
                "gasfm_edge_seam_fwd: aligned rows required");
  GASFM_REQUIRE(slope >= 0.f && slope <= 1.f, "gasfm_edge_seam_fwd: negative_slope %g outside [0, 1]", double(slope));
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const SeamEpi ep{Pb, P0, pt, ln_wb, ln_bb, eps_b, Wp, ldWp, bp, Sp, Sv, ldSv, Sg, scale, Pout,
                   nullptr, nullptr, nullptr, nullptr};
  auto launch = [&](auto kern) {
    const int grid = resident_grid(reinterpret_cast<const void*>(kern), kThreads, 0, n_items, kWaves);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, ep, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, ldXLp,
                       pos, XR, ldXR, att, bias, slope, items, n_items, finalize, out, ldOut, seg_max, seg_sum,
                       ldStat, part);
  };
  note_dispatch(GASFM_K_SEAM_REG);
  if (ln_w)
    launch(&edge_seam_fwd_kernel<true, false>);
  else
    launch(&edge_seam_fwd_kernel<false, false>);
  return launch_status("gasfm_edge_seam_fwd");
}

extern "C" int gasfm_edge0_seam_fwd(const float* P, const int32_t* pt, const float* ln_a_w, const float* ln_a_b,
                                    const float* ln_b_w, const float* ln_b_b, float eps0, const float* Wp,
                                    const float* bp, const float* Wsk, const float* bsk, const float* Sp,
                                    const float* Sv, int64_t ldSv, const float* Sg, float scale, float* Pout,
                                    const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                                    const float* bpt, const float* Wc, const float* bc, float* XLp, int64_t ldXLp,
                                    const int32_t* pos, const float* XR, int64_t ldXR, const float* att,
                                    const float* bias, float slope, const gasfm_work_item* items, int32_t n_items,
                                    int32_t finalize, float* out, int64_t ldOut, float* seg_max, float* seg_sum,
                                    int64_t ldStat, float* part, void* stream) {
  GASFM_REQUIRE(n_items >= 0 && P && pt && ln_a_w && ln_a_b && ln_b_w && ln_b_b && Wp && bp && Wsk && bsk && Sp &&
                    Sv && Sg && Pout && ln_w && ln_b && Wpt && bpt && Wc && bc && XLp && XR && att && items,
                "gasfm_edge0_seam_fwd: null pointer");
  GASFM_REQUIRE((out && seg_max && seg_sum && (bias || !finalize)) || part, "gasfm_edge0_seam_fwd: no outputs");
  GASFM_REQUIRE(ldXLp >= F && ldXLp % 4 == 0 && ldXR >= F && ldXR % 4 == 0 && ldSv >= F && ldSv % 4 == 0 &&
                    (!out || (ldOut >= F && ldOut % 4 == 0)) && reinterpret_cast<uintptr_t>(P) % 8 == 0 &&
                    aligned16(Pout) && aligned16(Sp) && aligned16(Sv) && aligned16(XLp) && aligned16(XR) &&
                    (!out || aligned16(out)) && (!part || aligned16(part)),
                "gasfm_edge0_seam_fwd: aligned rows required");
  GASFM_REQUIRE(slope >= 0.f && slope <= 1.f, "gasfm_edge0_seam_fwd: negative_slope %g outside [0, 1]", double(slope));
  if (n_items == 0) return GASFM_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const SeamEpi ep{P, nullptr, pt, ln_a_w, ln_a_b, eps0, Wp, 2, bp, Sp, Sv, ldSv, Sg, scale, Pout,
                   ln_b_w, ln_b_b, Wsk, bsk};
  const auto kern = &edge_seam_fwd_kernel<true, true>;
  const int grid = resident_grid(reinterpret_cast<const void*>(kern), kThreads, 0, n_items, kWaves);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, st, ep, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, ldXLp, pos,
                     XR, ldXR, att, bias, slope, items, n_items, finalize, out, ldOut, seg_max, seg_sum, ldStat, part);
  return launch_status("gasfm_edge0_seam_fwd");
}
