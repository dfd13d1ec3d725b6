/*
 * gasfm.h — C ABI of the MI355X (gfx950) GASFM graph-attention hot path.
 *
 * The reference has no native boundary for this path: the arithmetic sits in
 * PyG's GATv2Conv (third party, called at code/models/layers.py:329-335,
 * 426-432, 550-556, 566-572) and in aten ops inside
 * GraphAttnSfMLayer / GraphAttnSfMProjectionFeatureUpdate
 * (layers.py:222-263, 911-956).  Each entry point below names the reference
 * computation it replaces.  The Python host side (gasfm_amd/) binds these
 * through ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Plain pointers and sizes; no torch types.  All device buffers are
 *    caller-allocated (the library never allocates device memory), fp32
 *    features, int32 indices, row-major with explicit leading dimensions
 *    (in elements; feature row starts must be 16-byte aligned).
 *  - `stream` is a hipStream_t passed as void* (the caller's current stream).
 *  - Every function returns a status code (GASFM_OK == 0) and never aborts;
 *    gasfm_last_error() returns a thread-local message for the last failure.
 *    GASFM_ERR_OOM corresponds to hipErrorOutOfMemory (host maps it to
 *    torch.OutOfMemoryError, which train.py:225-241 catches).
 *  - Reductions are deterministic: no float atomics anywhere; segment sums
 *    are done by one wave per segment piece plus ordered combine passes.
 */
#ifndef GASFM_H
#define GASFM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  GASFM_OK = 0,
  GASFM_ERR_INVALID = 1,     /* bad argument / shape / alignment */
  GASFM_ERR_OOM = 2,         /* hipErrorOutOfMemory */
  GASFM_ERR_HIP = 3,         /* any other HIP runtime error */
  GASFM_ERR_UNSUPPORTED = 4  /* (H, C) combination without a kernel */
};

/* One unit of attention work: edges [begin, end) (positions in the segment's
 * edge order, i.e. indices into `perm` when perm != NULL) of segment `seg`.
 * slot < 0: the item covers the whole segment and writes the segment's
 * result directly; slot >= 0: it writes an un-normalised partial
 * (max, sum, acc) into partial slot `slot`. */
typedef struct gasfm_work_item {
  int32_t seg, begin, end, slot;
} gasfm_work_item;

/* Ordered combine of partial slots: slots slot_begin + k*slot_stride,
 * k = 0..slot_count-1, are merged (in k order) into segment `seg`. */
typedef struct gasfm_combine_item {
  int32_t seg, slot_begin, slot_count, slot_stride;
} gasfm_combine_item;

const char* gasfm_last_error(void);
int gasfm_version(void);

/* ---- kernel-choice record and tuning (host) ----------------------------- */

/* Kernels picked by the size / occupancy dependent dispatches.  Every launch
 * through such a dispatch bumps its counter at launch time (a captured graph
 * counts once per capture).  Test and profiling infrastructure only: the
 * reference has no counterpart. */
enum {
  GASFM_K_ATTN_FWD_GRP = 0,      /* grouped items, 8 segments per wave task (32-wide, streamed XL) */
  GASFM_K_ATTN_FWD_GLDS = 1,     /* one item per wave, direct-to-LDS prefetch (32-wide, streamed) */
  GASFM_K_ATTN_FWD_VEC = 2,      /* one item per wave, registers (any tabulated (H, C), perm ok) */
  GASFM_K_ATTN_FWD_GENERIC = 3,  /* any (H, C) */
  GASFM_K_ATTN_FWD_LANES = 4,    /* one lane per item (H = 4, C = 1) */
  GASFM_K_ATTN_BWD_GLDS = 5,
  GASFM_K_ATTN_BWD_VEC = 6,
  GASFM_K_ATTN_BWD_GENERIC = 7,
  GASFM_K_ATTN_BWD_LANES = 8,
  GASFM_K_ATTN_COMBINE_VEC = 9,
  GASFM_K_ATTN_COMBINE_GENERIC = 10,
  /* 11, 12: reserved (round-4 variants measured and removed: grouped attention backward,
   * LDS-staged forward seam); 14 was the grouped segment row sums */
  GASFM_K_SEAM_REG = 13,         /* forward seam (blocks 1-11) */
  GASFM_K_ATTN_FWD_GRP_S2 = 14,  /* grouped items, 2 lane groups per item (also counted as _GRP) */
  GASFM_K_ATTN_FWD_GRP_S4 = 15,  /* grouped items, 4 lane groups per item (also counted as _GRP) */
  GASFM_K_COUNT = 16
};

/* Copies min(n, GASFM_K_COUNT) counters into out; returns GASFM_K_COUNT. */
int gasfm_dispatch_counts(int64_t* out, int32_t n);
void gasfm_dispatch_reset(void);

/* Dispatch thresholds (initialised from the environment variable named in
 * the comment; gasfm_tuning_set overrides them for the rest of the process). */
enum {
  GASFM_TUNE_ATTN_GRP_ROWS = 0,      /* GASFM_ATTN_GRP: 4 / 8 / 46 / 48, 0 = grouped forward off */
  GASFM_TUNE_ATTN_GRP_MIN_FILL = 1,  /* GASFM_ATTN_GRP_MIN_FILL: grouped when tasks >= fill x resident waves */
  GASFM_TUNE_ATTN_GLDS = 2,          /* GASFM_ATTN_GLDS: direct-to-LDS kernels on (1) / off (0) */
  GASFM_TUNE_ATTN_WAVE_CAP = 3,      /* GASFM_ATTN_WAVES: cap on item-loop waves, 0 = occupancy */
  GASFM_TUNE_ATTN_GRP_SPLIT = 4,     /* GASFM_ATTN_SPLIT: lane groups per item of the grouped forward, 1 / 2 / 4;
                                        0 = by size: 2 when the 1-group tasks fit in the resident waves */
  /* 5, 6: reserved (removed round-4 variants) */
  GASFM_TUNE_COUNT = 8
};
int gasfm_tuning_set(int32_t key, double value);
double gasfm_tuning_get(int32_t key);

/* ---- graph preprocessing (host, CPU; usable in DataLoader workers) ------ */

/* Counting-sort CSR build: ptr[n+1] = segment offsets of `key` (values in
 * [0, n)), perm[E] = edge ids grouped by key, stable (ascending edge id inside
 * a segment).  Replaces the implicit grouping PyG's scatter does over
 * edge_index[1] (dataset_utils.py:531-535) for the unsorted point direction.
 * Reference-side caller: SceneData.create_axial_aggregation_graphs
 * (SceneData.py:153-239). */
int gasfm_build_csr(const int32_t* key, int64_t E, int32_t n,
                    int32_t* ptr, int32_t* perm);

/* Split segments longer than max_piece edges into pieces.  Writes at most
 * *n_items items (capacity in, count out) and *n_combine combine entries;
 * returns GASFM_ERR_INVALID if a capacity is too small (counts then hold the
 * required sizes).  all_partial != 0 makes every segment write a partial
 * (multi-GPU camera direction), with slot == seg for unsplit segments. */
int gasfm_plan_work(const int32_t* seg_ptr, int32_t N, int32_t max_piece,
                    int32_t all_partial,
                    gasfm_work_item* items, int32_t* n_items,
                    gasfm_combine_item* combine, int32_t* n_combine,
                    int32_t* n_slots);

/* ---- edge prologue + camera-direction attention (device, edge_cam.hip) --
 * One pass over the camera plan's work items (contiguous edges of one camera) replaces
 * gasfm_edge_prologue_fwd + gasfm_gat_attn_fwd on the camera half of XL (the lin_l of both convs,
 * layers.py:232-234 + PyG; Proj2View's attention, layers.py:329-335): XLp [E, 32] = Wpt
 * relu(LN(P)) + bpt is written (row pos[e] when pos != NULL, else row e), XLc = Wc relu(LN(P)) + bc
 * is consumed in registers, and the camera aggregates are written exactly as gasfm_gat_attn_fwd
 * writes them for these items (H = 4, C = 8; out / seg_max / seg_sum, or packed partial rows of
 * 40 floats).  ln_w == NULL: no LayerNorm (the final update's raw features). */
int gasfm_edge_cam_fwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                       const float* bpt, const float* Wc, const float* bc, float* XLp, int64_t ldXLp,
                       const int32_t* pos, const float* XR, int64_t ldXR, const float* att, const float* bias,
                       float slope, const gasfm_work_item* items, int32_t n_items, int32_t finalize, float* out,
                       int64_t ldOut, float* seg_max, float* seg_sum, int64_t ldStat, float* part, void* stream);
/* Backward of the camera attention above (gasfm_gat_attn_bwd on these items) with XLc recomputed
 * from P instead of read: given the camera aggregates' gradient gout and the forward's out /
 * seg_max / seg_sum, writes dXLc [E, 32] (row stride ldD; gasfm_edge_prologue_bwd's camera half),
 * dXR[seg] for complete items (split items: part_dxr[slot], merge with
 * gasfm_gat_attn_bwd_combine) and one partial row per workgroup
 * part[gasfm_edge_cam_bwd_part_rows(n_items), gasfm_edge_cam_bwd_part_cols()] = [datt 32 | dbias 32]
 * (reduce with gasfm_colsum). */
int32_t gasfm_edge_cam_bwd_part_rows(int32_t n_items);
int32_t gasfm_edge_cam_bwd_part_cols(void);
int gasfm_edge_cam_bwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wc,
                       const float* bc, const float* XR, int64_t ldXR, const float* att, const float* bias,
                       float slope, const float* out, int64_t ldOut, const float* seg_max, const float* seg_sum,
                       int64_t ldStat, const float* gout, int64_t ldG, const gasfm_work_item* items,
                       int32_t n_items, float* dXLc, int64_t ldD, float* dXR, int64_t ldDXR, float* part_dxr,
                       float* part, void* stream);

/* Block b's edge epilogue and block b+1's edge prologue + camera-direction attention forward in ONE
 * pass over block b+1's camera plan items (gasfm_edge_epilogue_fwd of block b followed by
 * gasfm_edge_cam_fwd of block b+1 on its output, without reading that output back):
 *   Pout = Pb + scale (Wp [relu(LN_b(Pb)) | P0] + bp + Sp[pt] + Sv[cam] + Sg)   (stored)
 * and every output of gasfm_edge_cam_fwd for P = Pout (ln_w / ln_b: block b+1's LayerNorm, null =
 * none).  Replaces (reference): GraphAttnSfMProjectionFeatureUpdate + the residual of block b
 * (layers.py:911-956, 254-261) and block b+1's LayerNorm, lin_l and Proj2View GATv2Conv forward
 * (layers.py:232-234, 329-335). */
int gasfm_edge_seam_fwd(const float* Pb, const float* P0, const int32_t* pt, const float* ln_wb, const float* ln_bb,
                        float eps_b, const float* Wp, int32_t ldWp, const float* bp, const float* Sp, const float* Sv,
                        int64_t ldSv, const float* Sg, float scale, float* Pout, const float* ln_w,
                        const float* ln_b, float eps, const float* Wpt, const float* bpt, const float* Wc,
                        const float* bc, float* XLp, int64_t ldXLp, const int32_t* pos, const float* XR,
                        int64_t ldXR, const float* att, const float* bias, float slope,
                        const gasfm_work_item* items, int32_t n_items, int32_t finalize, float* out, int64_t ldOut,
                        float* seg_max, float* seg_sum, int64_t ldStat, float* part, void* stream);
/* Block 0's edge epilogue (2-wide P: P' = Wsk relu(LN_b(P)) + bsk + scale (Wp relu(LN_a(P)) + bp +
 * Sg + Sp[pt] + Sv[cam]), gasfm_edge0_epilogue_fwd) and block 1's prologue + camera attention
 * (gasfm_edge_cam_fwd) in ONE pass, as gasfm_edge_seam_fwd for the 32-wide blocks (round 3).
 * Replaces (reference): layers.py:245-261 / 911-956 of block 0 and 232-234, 329-335 of block 1. */
int gasfm_edge0_seam_fwd(const float* P, const int32_t* pt, const float* ln_a_w, const float* ln_a_b,
                         const float* ln_b_w, const float* ln_b_b, float eps0, const float* Wp, const float* bp,
                         const float* Wsk, const float* bsk, const float* Sp, const float* Sv, int64_t ldSv,
                         const float* Sg, float scale, float* Pout, const float* ln_w, const float* ln_b, float eps,
                         const float* Wpt, const float* bpt, const float* Wc, const float* bc, float* XLp,
                         int64_t ldXLp, const int32_t* pos, const float* XR, int64_t ldXR, const float* att,
                         const float* bias, float slope, const gasfm_work_item* items, int32_t n_items,
                         int32_t finalize, float* out, int64_t ldOut, float* seg_max, float* seg_sum, int64_t ldStat,
                         float* part, void* stream);

/* The camera attention's backward and the block's edge prologue backward in ONE pass over the
 * camera plan's items (gasfm_edge_cam_bwd followed by gasfm_edge_prologue_bwd with dXLc, without
 * storing dXLc): dP [E, 32], dXR per camera (split items: part_dxr rows for
 * gasfm_gat_attn_bwd_combine), and per workgroup the partial row
 * [dW 64x32 | db 64 | dgamma 32 | dbeta 32 | datt 32 | 0 (32)]; the attention bias gradient is the
 * column sum of gout over all targets (every target's output carries the bias), taken by the caller
 * (part[gasfm_edge_cam_pbwd_part_rows(n_items), gasfm_edge_cam_pbwd_part_cols()]).
 * dXLp: the point half of dXL in edge order (row stride ldXp); dRes / Wp (row stride ldWp) / scale:
 * the block output's residual gradient and lin_proj, as in gasfm_edge_prologue_bwd (dRes may be null).
 * Replaces (reference): the autograd of Proj2View's GATv2Conv and of the LayerNorm + lin_l on the
 * projection features (layers.py:232-234, 329-335). */
int32_t gasfm_edge_cam_pbwd_part_rows(int32_t n_items);
int32_t gasfm_edge_cam_pbwd_part_cols(void);
int gasfm_edge_cam_pbwd(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                        const float* Wc, const float* bc, const float* Wp, int32_t ldWp, float scale,
                        const float* XR, int64_t ldXR, const float* att, const float* bias, float slope,
                        const float* out, int64_t ldOut, const float* seg_max, const float* seg_sum,
                        int64_t ldStat, const float* gout, int64_t ldG, const gasfm_work_item* items,
                        int32_t n_items, const float* dXLp, int64_t ldXp, const float* dRes, float* dP,
                        float* dXR, int64_t ldDXR, float* part_dxr, float* part, void* stream);
/* gasfm_edge_cam_pbwd with the edge epilogue's backward folded in (round 3; replaces
 * gasfm_edge_epilogue_bwd's dSv / dP0 / dWp, reference: the autograd of lin_proj and of the
 * Sv[cam] gather in GraphAttnSfMProjectionFeatureUpdate, layers.py:911-956):
 *   dSv_e != null (EPI): the PREVIOUS block's epilogue gradients from this launch's dP (= that
 *     epilogue's dP'): dSv_e[cam] = scale_e sum_e dP[e] (split items: part_dsv_e rows, same slots as
 *     part_dxr), dP0_e[e] = scale_e We[:, 32:34]^T dP[e] (dP0_e may be null; We row stride ldWe);
 *     requires (ln_w == null) == (dRes == null);
 *   ldWpo > 0 (DWP): THIS block's lin_proj gradient scale sum_e dRes[e]^T [relu(LN(P[e])) | P0[e]]
 *     as a [32 x ldWpo] block after the gasfm_edge_cam_pbwd_part_cols() floats of each part row
 *     (ldWpo = 34 with P0 [E, 2], 32 without); requires ln_w and dRes.
 * part rows have stride ldPart (>= part_cols + 32 ldWpo). */
int gasfm_edge_cam_pbwd_ex(const float* P, const float* ln_w, const float* ln_b, float eps, const float* Wpt,
                           const float* Wc, const float* bc, const float* Wp, int32_t ldWp, float scale,
                           const float* XR, int64_t ldXR, const float* att, const float* bias, float slope,
                           const float* out, int64_t ldOut, const float* seg_max, const float* seg_sum,
                           int64_t ldStat, const float* gout, int64_t ldG, const gasfm_work_item* items,
                           int32_t n_items, const float* dXLp, int64_t ldXp, const float* dRes, float* dP,
                           float* dXR, int64_t ldDXR, float* part_dxr, float* part, int64_t ldPart,
                           const float* We, int32_t ldWe, float scale_e, float* dSv_e, float* part_dsv_e,
                           float* dP0_e, const float* P0, int32_t ldWpo, void* stream);

/* ---- fused GATv2 edge-softmax + aggregation (device) ------------------- */

/* Forward of PyG GATv2Conv's message/softmax/aggregate on pre-projected
 * rows (replaces gatv2_conv.py message() + utils.softmax + scatter 'add',
 * called at layers.py:329-335 etc.):
 *   e_j[h]   = sum_c att[h,c] * leaky_relu(XL[src_j,h,c] + XR[seg,h,c], slope)
 *   out[seg] = sum_j softmax_j(e)[h] * XL[src_j,h,:] + bias      (finalize)
 * src_j = perm[j] if perm != NULL else j.  Complete items (slot < 0) write
 * out[seg] (finalized if finalize != 0, otherwise the raw acc) plus
 * seg_max[seg*ldStat + h], seg_sum[seg*ldStat + h] (sum of exp(e - max), no
 * epsilon).  Items with slot >= 0 write a raw partial into the PACKED partial
 * row part[slot*(HC+2H) ..] = [acc (HC) | max (H) | sum (H)] — the unit one
 * rank contributes to the multi-GPU all-gather.  Segments with no edges give
 * out = bias, max = -inf, sum = 0. */
int gasfm_gat_attn_fwd(const float* XL, int64_t ldXL,
                       const float* XR, int64_t ldXR,
                       const float* att, const float* bias,
                       const int32_t* perm,
                       const gasfm_work_item* items, int32_t n_items,
                       int32_t H, int32_t C, float negative_slope,
                       int32_t finalize,
                       float* out, int64_t ldOut, float* seg_max, float* seg_sum, int64_t ldStat,
                       float* part, void* stream);

/* Ordered merge of packed partial rows (split pieces, or one row per rank
 * after an all-gather).  Writes out/seg_max/seg_sum at index seg: finalized
 * with bias when finalize != 0, else raw (pass out = a packed partial buffer,
 * ldOut = ldStat = HC+2H, seg_max = out+HC, seg_sum = out+HC+H). */
int gasfm_gat_attn_combine(const gasfm_combine_item* combine, int32_t n_combine,
                           int32_t H, int32_t C, const float* part,
                           const float* bias, int32_t finalize,
                           float* out, int64_t ldOut, float* seg_max, float* seg_sum,
                           int64_t ldStat, void* stream);

/* Lane-per-item variants of gasfm_gat_attn_fwd / _bwd for H = 4, C = 1 (block 0's 4-wide convs)
 * with short items (the point direction, ~20 edges per point): same arguments, outputs and
 * partial layouts; the backward's datt_part has gasfm_gat_attn_bwd_waves(n_items, 4, 1) rows. */
int gasfm_gat_attn_fwd_lanes(const float* XL, int64_t ldXL, const float* XR, int64_t ldXR, const float* att,
                             const float* bias, const int32_t* perm, const gasfm_work_item* items, int32_t n_items,
                             int32_t H, int32_t C, float slope, int32_t finalize, float* out, int64_t ldOut,
                             float* seg_max, float* seg_sum, int64_t ldStat, float* part, void* stream);
int gasfm_gat_attn_bwd_lanes(const float* XL, int64_t ldXL, const float* XR, int64_t ldXR, const float* att,
                             const float* bias, const int32_t* perm, const gasfm_work_item* items, int32_t n_items,
                             int32_t H, int32_t C, float slope, const float* out, int64_t ldOut,
                             const float* seg_max, const float* seg_sum, const float* gout, int64_t ldG, float* dXL,
                             int64_t ldDXL, float* dXR, int64_t ldDXR, float* part_dxr, float* datt_part,
                             int32_t xl_by_position, void* stream);

/* Backward of the above given dOut (gout), the forward's finalized out and
 * per-segment stats.  Writes dXL[src_j] for every edge (each row exactly
 * once), dXR[seg] for complete items (partials to part_dxr[slot] for split
 * items; merge with gasfm_gat_attn_bwd_combine) and one partial row per
 * wave into datt_part[n_waves, 2*H*C] = [d att | d bias] (n_waves from
 * gasfm_gat_attn_bwd_waves(), which sizes the grid from the current device's
 * occupancy for this (H, C); reduce with gasfm_colsum).  xl_by_position != 0:
 * XL rows are stored in segment order (row j, as the forward reads them with
 * perm = NULL) while dXL is still written at row perm[j] (edge order). */
int gasfm_gat_attn_bwd_waves(int32_t n_items, int32_t H, int32_t C);
int gasfm_gat_attn_bwd(const float* XL, int64_t ldXL,
                       const float* XR, int64_t ldXR,
                       const float* att, const float* bias,
                       const int32_t* perm,
                       const gasfm_work_item* items, int32_t n_items,
                       int32_t H, int32_t C, float negative_slope,
                       const float* out, int64_t ldOut,
                       const float* seg_max, const float* seg_sum,
                       const float* gout, int64_t ldG,
                       float* dXL, int64_t ldDXL,
                       float* dXR, int64_t ldDXR,
                       float* part_dxr, float* datt_part,
                       int32_t xl_by_position, void* stream);

/* dXR[seg] = sum_k part_dxr[slot_begin + k*slot_stride]  (ordered). */
int gasfm_gat_attn_bwd_combine(const gasfm_combine_item* combine, int32_t n_combine,
                               int32_t HC, const float* part_dxr,
                               float* dXR, int64_t ldDXR, void* stream);
/* gasfm_gat_attn_bwd_combine for two partial-row arrays over the same combine entries in ONE launch
 * (round 5: the camera plan's dXR and the folded epilogue's dSv rows, gasfm_edge_cam_pbwd_ex). */
int gasfm_gat_attn_bwd_combine2(const gasfm_combine_item* combine, int32_t n_combine, int32_t HC,
                                const float* part_a, float* out_a, int64_t ld_a, const float* part_b,
                                float* out_b, int64_t ld_b, void* stream);

/* out[c] = sum_r A[r*ld + c] for c < cols: ONE launch, deterministic (per-block partial slabs
 * in ws, summed in block order by the last block of each column chunk).  ws must hold
 * gasfm_colsum_ws_floats(rows, cols) floats; counters must hold gasfm_colsum_counters(cols)
 * uint32 that are ZERO before the first call (the kernel resets them; one array per device,
 * calls ordered on one stream). */
int64_t gasfm_colsum_ws_floats(int64_t rows, int32_t cols);
int32_t gasfm_colsum_counters(int32_t cols);
int gasfm_colsum(const float* A, int64_t rows, int32_t cols, int64_t ld,
                 float* ws, float* out, uint32_t* counters, void* stream);

/* n independent colsums (job i: A[i] rows[i] x cols[i], row stride ld[i], workspace ws[i] of
 * gasfm_colsum_ws_floats(rows[i], cols[i]) floats, result out[i]) in ONE launch per 48 jobs;
 * counters: gasfm_colsum_multi_counters(n, cols) zeroed uint32 (self-resetting, shared with
 * gasfm_colsum: one array per device, calls ordered on one stream).  Same per-job results,
 * bit for bit, as gasfm_colsum.  Used for the weight-gradient partials of a backward pass. */
int gasfm_colsum_multi(int32_t n, const float* const* A, const int64_t* rows, const int32_t* cols,
                       const int64_t* ld, float* const* ws, float* const* out, uint32_t* counters,
                       void* stream);
int32_t gasfm_colsum_multi_counters(int32_t n, const int32_t* cols);

/* Column sums of a CONTIGUOUS tall, narrow [rows, cols] matrix (bias gradients over E edge or n
 * point rows), read as a flat coalesced stream: ONE launch, deterministic, up to 1024
 * workgroups.  Valid when gasfm_colsum_tall_ok(cols) (cols <= 256 and lcm(cols, 256) <= 2048).
 * ws: gasfm_colsum_tall_ws_floats(rows, cols) floats; counter: ONE zeroed uint32 (reset by
 * the kernel; calls ordered on one stream).  Replaces torch's global sum reduction, whose
 * replays inside a captured hipGraph were measured wrong. */
int32_t gasfm_colsum_tall_ok(int32_t cols);
int64_t gasfm_colsum_tall_ws_floats(int64_t rows, int32_t cols);
int gasfm_colsum_tall(const float* A, int64_t rows, int32_t cols, float* ws, float* out,
                      uint32_t* counter, void* stream);

/* ---- fused per-edge block body (F = n_feat_proj = 32; XL width 64 = point|camera) ---- */

/* Floats of the per-workgroup partial buffer: which = 0 -> edge_prologue_bwd
 * ([64*32 dW | 64 db | 32 dgamma | 32 dbeta] per workgroup), 1 -> edge_epilogue_bwd
 * ([32*34 dWp] per workgroup).  Reduce with gasfm_colsum. */
int gasfm_edge_part_floats(int32_t which, int64_t E, int32_t n_items);

/* XL[e] = W relu(LN(P[e])) + b  (ln_w == NULL: XL[e] = W P[e] + b, the final update).
 * Replaces LayerNorm+ReLU (layers.py:232-234) and both GATv2 lin_l on the edge rows
 * (layers.py:329, 426; PyG evaluates them on all E+N rows). W = [Wl_point; Wl_camera] [64x32].
 * pos != NULL: the point half (columns 0..31) of edge e is written to row pos[e] (its position
 * in point-segment order), so the point-direction attention streams it (perm = NULL forward,
 * xl_by_position backward); the camera half stays at row e. */
int gasfm_edge_prologue_fwd(const float* P, int64_t E, const float* ln_w, const float* ln_b, float eps,
                            const float* W, const float* W2, const float* b, const float* b2, float* Y,
                            int64_t ldY, const int32_t* pos, void* stream);

/* P'[e] = P[e] + scale*(Wp [relu(LN(P[e])) | P0[e]] + bp + Sp[pt[e]] + Sv[cam[e]] + Sg)
 * (GraphAttnSfMProjectionFeatureUpdate.forward, layers.py:927-945, + residual 254-261;
 * scale = 1/4).  Wp [32 x ldWp], ldWp = 34 with P0 [E x 2], 32 without.  Sv rows are ldSv
 * floats apart (32, or 64 when Sv is the first half of a gathered [SV | XR] row block). */
int gasfm_edge_epilogue_fwd(const float* P, const float* P0, const int32_t* cam, const int32_t* pt,
                            int64_t E, const float* ln_w, const float* ln_b, float eps,
                            const float* Wp, int32_t ldWp, const float* bp, const float* Sp,
                            const float* Sv, int64_t ldSv, const float* Sg, float scale, float* Pout,
                            void* stream);

/* Backward of the epilogue's reductions over the camera work items (contiguous
 * edges of one camera): dSv[cam] (partials to part_dsv for split items),
 * dP0 [E x 2], per-workgroup dWp partials.  Replaces the index_add scatter of
 * view_features[cam] (layers.py:940) and the K=E weight-gradient GEMM of lin_proj. */
int gasfm_edge_epilogue_bwd(const gasfm_work_item* items, int32_t n_items, const float* dPo,
                            const float* P, const float* P0, const float* ln_w, const float* ln_b,
                            float eps, const float* Wp, int32_t ldWp, float scale, float* dSv,
                            float* part_dsv, float* dP0, float* part_w, void* stream);

/* dP = LN_bwd(relu_mask * (W^T dXL + scale*Wp[:, :32]^T dRes)) + dRes, and the
 * per-workgroup partials of dW, db, dgamma, dbeta (LayerNorm/ReLU/lin_l backward).
 * dXLc != NULL: dXL holds only the point half ([E, >= 32], row stride ldX) and dXLc the camera
 * half ([E, >= 32], row stride ldC), as gasfm_edge_cam_bwd writes it. */
int gasfm_edge_prologue_bwd(const float* dXL, int64_t ldX, const float* P, const float* dRes,
                            int64_t E, const float* ln_w, const float* ln_b, float eps,
                            const float* W, const float* W2, const float* Wp, int32_t ldWp,
                            float scale, float* dP, float* part, const float* dXLc, int64_t ldC,
                            void* stream);

/* out[seg] = scale * sum_{edges of the item} X[src]  (32-wide rows; src via perm).
 * Replaces the index_add scatter of scenepoint_features[pt] (layers.py:940). */
int gasfm_segment_rowsum(const gasfm_work_item* items, int32_t n_items, const int32_t* perm,
                         const float* X, int64_t ldX, float scale, float* out, float* part,
                         void* stream);

/* ---- block 0 per-edge body (2-wide embedded projections; layers.py:148-263 with F_in = 2) ---- */

/* Partial rows per workgroup: which = 0 -> edge0_prologue_bwd ([dW0 16 | db0 8 | dgamma_a 2 |
 * dbeta_a 2]), 1 -> edge0_epilogue_bwd ([dWp 64 | dWsk 64 | dbsk 32 | dgamma_b 2 | dbeta_b 2]). */
int gasfm_edge0_part_rows(int32_t which, int64_t E, int32_t n_items);

/* XL0[e] (8 floats) = W0 relu(LN_a(P[e])) + b0, W0 = [Wl_point; Wl_camera] [8 x 2].
 * pos != NULL: the point half (4 floats) goes to row pos[e] (point-segment order), as in
 * gasfm_edge_prologue_fwd. */
int gasfm_edge0_prologue_fwd(const float* P, int64_t E, const float* ln_w, const float* ln_b, float eps,
                             const float* W0, const float* b0, float* XL, const int32_t* pos, void* stream);

/* The same XL0 (bitwise) written row by row: row r = [point half of edge perm[r] | camera half of
 * edge r], perm = the point plan's permutation (the inverse of pos above), so every row is one
 * contiguous 32-B store instead of a scattered 16-B point half. */
int gasfm_edge0_prologue_fwd_rows(const float* P, int64_t E, const float* ln_w, const float* ln_b, float eps,
                                  const float* W0, const float* b0, float* XL, const int32_t* perm,
                                  void* stream);

/* P'[e] = Wsk relu(LN_b(P[e])) + bsk + scale*(Wp relu(LN_a(P[e])) + bp + Sp[pt] + Sv[cam] + Sg). */
int gasfm_edge0_epilogue_fwd(const float* P, const int32_t* cam, const int32_t* pt, int64_t E,
                             const float* ln_a_w, const float* ln_a_b, const float* ln_b_w,
                             const float* ln_b_b, float eps, const float* Wp, const float* bp,
                             const float* Wsk, const float* bsk, const float* Sp, const float* Sv,
                             int64_t ldSv, const float* Sg, float scale, float* Pout, void* stream);

/* Camera work items: dSv (+ partial slots), aux[e] = (dP_hat_a (2), dP from the skip branch (2)),
 * per-workgroup partials of dWp, dWsk, dbsk, dgamma_b, dbeta_b. */
int gasfm_edge0_epilogue_bwd(const gasfm_work_item* items, int32_t n_items, const float* dPo,
                             const float* P, const float* ln_a_w, const float* ln_a_b,
                             const float* ln_b_w, const float* ln_b_b, float eps, const float* Wp,
                             const float* Wsk, float scale, float* dSv, float* part_dsv, float* aux,
                             float* part, void* stream);

/* dP = LN_a_bwd(mask (W0^T dXL0 + aux.xy)) + aux.zw and partials of dW0, db0, dgamma_a, dbeta_a. */
int gasfm_edge0_prologue_bwd(const float* dXL, const float* P, const float* aux, int64_t E,
                             const float* ln_w, const float* ln_b, float eps, const float* W0, float* dP,
                             float* part, void* stream);

/* ---- point-node rows: LayerNorm -> ReLU -> Linear (-> + x), n_in = 64, n_out in {32, 64} ----
 * Replaces the aten chains on the scene-point features (n rows x n_feat_scenepoint):
 * the state projection Sequential(LayerNorm, ReLU, Linear) (layers.py:48-56, used at
 * layers.py:403-404), the pre-MLP skip x + mlp(relu(norm_pre_mlp(x))) (layers.py:449-456) and
 * lin_scenepoint(relu(scenepoint_norm_layer(x))) of the projection update (layers.py:928-935). */

/* Rows of the [rows x (n_out*n_in + n_out + 2*n_in)] partial buffer gasfm_node_ln_linear_bwd
 * writes for this (N, n_out, residual): [dW n_out x n_in | db n_out | dgamma n_in | dbeta n_in]
 * per workgroup (the grid is sized to the resident workgroups of the current device). */
int gasfm_node_part_rows(int64_t N, int32_t n_out, int32_t residual);

/* Y[i] = W relu(LN(X[i])) + b (+ X[i] if residual); b may be null. X: [N x 64] contiguous. */
int gasfm_node_ln_linear_fwd(const float* X, int64_t N, int32_t n_in, const float* ln_w, const float* ln_b,
                             float eps, const float* W, const float* b, int32_t n_out, int32_t residual,
                             float* Y, int64_t ldY, void* stream);

/* dX = LN_bwd(mask * (dY W)) (+ dY if residual) and the per-workgroup partials above. */
int gasfm_node_ln_linear_bwd(const float* dY, const float* X, int64_t N, int32_t n_in, const float* ln_w,
                             const float* ln_b, float eps, const float* W, int32_t n_out, int32_t residual,
                             float* dX, float* part, void* stream);

/* ---- scene-point block chains (n rows x 64; aggregation / projection width 32) ----
 * tail: the end of Proj2ScenePoint.forward (layers.py:438-454)
 *   x = prev + Wp agg + bp ; p = x + Wm relu(LN(x)) + bm          (prev may be null: block 0)
 * hub: every consumer of p in one pass --
 *   SA = WA relu(LN_A(p))           lin_scenepoint(relu(scenepoint_norm_layer(p))) (layers.py:928-935)
 *   XL = WB p + bB                  graph_conv_scenepoint2global.lin_l (PyG, layers.py:560-575)
 *   XR = WD (WC relu(LN_C(p)) + bWC) + bD    the next block's norm_and_proj_scenepoint2proj
 *                                   (layers.py:429) and its graph_conv.lin_r; gC == null skips it
 * Backward gradients of weights / biases / LayerNorm affines leave as per-workgroup partial
 * rows ([rows x cols], shapes from the *_part_shape queries) for gasfm_colsum. */

/* Partial buffer rows for gasfm_point_tail_bwd; *cols receives the row width:
 * [dWm 64x64 | dWp 64x32 | dbm 64 | dbp 64 | dgamma 64 | dbeta 64]. */
int gasfm_point_tail_part_shape(int64_t N, int32_t has_prev, int32_t* cols);

/* Partial buffer rows for gasfm_point_hub_bwd_ab (which = 0):
 *   [dWA 32x64 | dWB 64x64 | dbB 64 | dgamma_A 64 | dbeta_A 64]
 * or gasfm_point_hub_bwd_c (which = 1):
 *   [dWC 32x64 | dWD 32x32 | dbWC 32 | dbD 32 | dgamma_C 64 | dbeta_C 64]. */
int gasfm_point_hub_part_shape(int64_t N, int32_t which, int32_t has_res, int32_t* cols);

int gasfm_point_tail_fwd(const float* prev, const float* agg, int64_t N, const float* Wp, const float* bp,
                         const float* ln_w, const float* ln_b, float eps, const float* Wm, const float* bm,
                         float* out, void* stream);

/* dx = dout + LN_bwd(mask (dout Wm)) (== d prev), dagg = dx Wp, partials. */
int gasfm_point_tail_bwd(const float* dout, const float* prev, const float* agg, int64_t N, const float* Wp,
                         const float* bp, const float* ln_w, const float* ln_b, float eps, const float* Wm,
                         float* dx, float* dagg, float* part, void* stream);

int gasfm_point_hub_fwd(const float* X, int64_t N, float eps, const float* gA, const float* bA, const float* WA,
                        float* SA, const float* WB, const float* bB, float* XL, const float* gC, const float* bC,
                        const float* WC, const float* bWC, const float* WD, const float* bD, float* XR,
                        void* stream);

/* gasfm_point_tail_fwd then gasfm_point_hub_fwd on its output in ONE launch (round 6): out = p, and
 * SA / XL / (gC non-null) XR of p, bitwise as the two calls; eps_h: the hub's LayerNorm epsilon.
 * Replaces the pair the reference runs as Proj2ScenePoint's tail (code/models/layers.py:438-454) and
 * the consumers of its output (:429, :560-575, :924-935). */
int gasfm_point_tail_hub_fwd(const float* prev, const float* agg, int64_t N, const float* Wp, const float* bp,
                             const float* ln_w, const float* ln_b, float eps, const float* Wm, const float* bm,
                             float* out, float eps_h, const float* gA, const float* bA, const float* WA, float* SA,
                             const float* WB, const float* bB, float* XL, const float* gC, const float* bC,
                             const float* WC, const float* bWC, const float* WD, const float* bD, float* XR,
                             void* stream);

/* dX = dRes + LN_C_bwd(mask (dXR WD WC)) (dRes may be null), partials. */
int gasfm_point_hub_bwd_c(const float* X, int64_t N, float eps, const float* gC, const float* bC, const float* WC,
                          const float* bWC, const float* WD, const float* dXR, const float* dRes, float* dX,
                          float* part, void* stream);

/* dX = dRes + dXL WB + LN_A_bwd(mask (dSA WA)) (dRes may be null), partials. */
int gasfm_point_hub_bwd_ab(const float* X, int64_t N, float eps, const float* gA, const float* bA,
                           const float* WA, const float* WB, const float* dSA, const float* dXL,
                           const float* dRes, float* dX, float* part, void* stream);

/* The whole hub backward in one pass (both of the above; the two-pass form when the library is
 * built with GASFM_PT_HUB_BWD_R=0): dX = dRes + dXL WB + LN_A_bwd(mask (dSA WA))
 * + LN_C_bwd(mask (dXR WD WC)); dRes may be null or alias dX, dX must not alias the other inputs.
 * part_a / part_c: the which = 0 / which = 1 partial layouts above, gasfm_point_hub_part_shape rows. */
int gasfm_point_hub_bwd(const float* X, int64_t N, float eps, const float* gA, const float* bA, const float* WA,
                        const float* WB, const float* gC, const float* bC, const float* WC, const float* bWC,
                        const float* WD, const float* dSA, const float* dXL, const float* dXR, const float* dRes,
                        float* dX, float* part_a, float* part_c, void* stream);

/* ---- input embedding (embed.hip): P = values W^T + b, the Linear(2, 2) of EmbeddingLayer
 * (layers.py:992-1015, graph_attn_sfm.py:53); values, P [E x 2] row-major, W [2 x 2], b [2]. */
int gasfm_embed2_fwd(const float* values, int64_t E, const float* W, const float* b, float* P, void* stream);
/* Partial rows (6 floats: dW00 dW01 dW10 dW11 db0 db1) of gasfm_embed2_bwd; their column sums
 * are dW and db. */
int32_t gasfm_embed2_part_rows(int64_t E);
int gasfm_embed2_bwd(const float* values, const float* dP, int64_t E, float* part, void* stream);

/* ---- scene-point head (point_head.hip): replaces the aten run of
 *   pts3D = [scenepoint_head(relu(p))^T ; 1]   (graph_attn_sfm.py:170-174, layers.py:10-44,
 *   norm=False, 2 hidden layers: Linear(64,64) ReLU Linear(64,64) ReLU Linear(64,3)).
 * P [N x 64] row-major; W1, W2 [64 x 64], W3 [3 x 64] (torch Linear [out, in]); out / dout [4 x N]. */

/* Partial rows for gasfm_point_head_bwd: which = 0 -> part_a [dW1 64x64 | db1 64],
 * which = 1 -> part_b [dW2 64x64 | dW3 3x64 | db2 64 | db3 3]; *cols receives the row width. */
int gasfm_point_head_part_shape(int64_t N, int32_t which, int32_t* cols);

/* out[0:3] = (relu(relu(relu(P) W1^T + b1) W2^T + b2) W3^T + b3)^T, out[3] = 1. */
int gasfm_point_head_fwd(const float* P, int64_t N, const float* W1, const float* b1, const float* W2,
                         const float* b2, const float* W3, const float* b3, float* out, void* stream);

/* dP and the weight-gradient partials (column sums give dW1, db1, dW2, dW3, db2, db3) from
 * dout rows 0-2 (row 3, the constant ones, has no gradient). */
int gasfm_point_head_bwd(const float* P, int64_t N, const float* W1, const float* b1, const float* W2,
                         const float* b2, const float* W3, const float* dout, float* dP, float* part_a,
                         float* part_b, void* stream);

/* ---- camera (view) block chains (m rows x D, D a multiple of 64, <= 1024) ----
 * tail: Proj2View.forward after the aggregation (layers.py:345-360):
 *   x = prev + Wp agg + bp;  view = x + Wm relu(LN(x)) + bm
 *   gasfm_view_tail_fwd writes x, xb = x + bm, h = relu(LN(x)) and the row (mean, rstd) of x
 *   (rs, m x 2); the caller's GEMM computes view = xb + h Wm^T (hipBLASLt).
 * hub: SV = Wv relu(LN_c(v)) (lin_view, layers.py:928-935), T = Wa relu(LN_a(v)) + ba and
 *   XR = Wr T + br (the next block's norm_and_proj_view2proj + lin_r), row (mean, rstd) of v;
 *   the caller's GEMM computes graph_conv_view2global.lin_l(v).
 * Every kernel runs one wave per (16-row tile, 64-column block); whole-row quantities cross the
 * column blocks through `scratch` (gasfm_view_scratch_floats(m, D) floats, caller-allocated).
 * Gradients of weights / biases / LayerNorm affines leave as one partial row per tile
 * (ceil(m/16) rows) for gasfm_colsum. */

/* Partial-row widths: tail [dWp D x 32 | dbp D | dgamma D | dbeta D | dbm D];
 * hub [dWv 32 x D | dWa 32 x D | dgamma_c | dbeta_c | dgamma_a | dbeta_a | dbl (each D) |
 *      dWr 32 x 32 | dba 32 | dbr 32]. */
int gasfm_view_tail_part_cols(int32_t D);
int gasfm_view_hub_part_cols(int32_t D);
int64_t gasfm_view_scratch_floats(int64_t m, int32_t D);

int gasfm_view_tail_fwd(const float* prev, const float* agg, int64_t m, int32_t D, const float* Wp, const float* bp,
                        const float* ln_w, const float* ln_b, float eps, const float* bm, float* x, float* xb,
                        float* h, float* rs, float* scratch, void* stream);

/* dx = dv + LN_bwd(mask dh) (dh = dv Wm from the caller's GEMM; == d prev), dagg = dx Wp, partials. */
int gasfm_view_tail_bwd(const float* dv, const float* dh, const float* x, const float* rs, const float* agg,
                        int64_t m, int32_t D, const float* Wp, const float* ln_w, const float* ln_b, float* dx,
                        float* dagg, float* part, float* scratch, void* stream);

/* sv and xr rows are ldo floats apart (32; 64 writes them side by side as one [m x 64] block,
 * the camera-sharded path's all-gather payload); t is [m x 32]. */
int gasfm_view_hub_fwd(const float* v, int64_t m, int32_t D, float eps, const float* gC, const float* bC,
                       const float* Wv, const float* gA, const float* bA, const float* Wa, const float* ba,
                       const float* Wr, const float* br, float* sv, float* t, float* xr, int32_t ldo, float* rs,
                       float* scratch, void* stream);

/* dacc (in: dXL Wl, out: d v) += dres + LN_c_bwd(mask dsv Wv) + LN_a_bwd(mask dt Wa), dt = dxr Wr;
 * dres (d skip, may be null) is added in the same pass (no addmm input copy); dxl is read for the
 * lin_l bias gradient; partials. */
int gasfm_view_hub_bwd(const float* v, const float* rs, int64_t m, int32_t D, const float* gC, const float* bC,
                       const float* Wv, const float* gA, const float* bA, const float* Wa, const float* t,
                       const float* Wr, const float* dsv, const float* dxr, const float* dxl, const float* dres,
                       float* dacc, float* part, float* scratch, void* stream);

/* ---- the camera side for SMALL row counts (view_chain.hip, round 4) ----
 * A camera-sharded rank's own rows (m / W) or a training batch's cameras: the same arithmetic as
 * gasfm_view_tail_* / gasfm_view_hub_* plus the D x D products they leave to a GEMM (Proj2View's
 * mlp, layers.py:345-360; graph_conv_view2global.lin_l, layers.py:551-556), with the GEMMs carrying
 * the view kernels as prologue / epilogue: 2 launches forward, 4 backward per block.  Applies
 * when gasfm_view_chain_ok(m, D): m <= 256, D in {256, 512, 1024}.  Parameter partial rows use
 * the gasfm_view_tail_part_cols / gasfm_view_hub_part_cols layouts. */
int32_t gasfm_view_chain_ok(int64_t m, int32_t D);
int64_t gasfm_view_chain_scratch_floats(int64_t m, int32_t D);
int32_t gasfm_view_chain_counters(int64_t m);
/* view = x + bm + relu(LN(x)) Wm^T, x = prev + agg Wp^T + bp; saves x, h = relu(LN(x)), rs. */
int gasfm_view_chain_tail_fwd(const float* prev, const float* agg, int64_t m, int32_t D, const float* Wp,
                              const float* bp, const float* ln_w, const float* ln_b, float eps, const float* Wm,
                              const float* bm, float* view, float* x, float* h, float* rs, void* stream);
/* XL = v Wl^T + bl; sv = relu(LN_c v) Wv^T; t = relu(LN_a v) Wa^T + ba; xr = t Wr^T + br (sv / xr
 * row stride ldo); rs = row (mean, rstd) of v. */
int gasfm_view_chain_hub_fwd(const float* v, int64_t m, int32_t D, float eps, const float* Wl, const float* bl,
                             const float* gC, const float* bC, const float* Wv, const float* gA, const float* bA,
                             const float* Wa, const float* ba, const float* Wr, const float* br, float* XL, float* sv,
                             float* t, float* xr, int32_t ldo, float* rs, void* stream);
/* dacc = d v = dres + dxl Wl + LN_c_bwd(mask dsv Wv) + LN_a_bwd(mask (dxr Wr) Wa); dWl = dxl^T v;
 * the other parameter gradients as partial rows. */
int gasfm_view_chain_hub_bwd(const float* v, const float* rs, int64_t m, int32_t D, const float* gC, const float* bC,
                             const float* Wv, const float* gA, const float* bA, const float* Wa, const float* t,
                             const float* Wr, const float* Wl, const float* dsv, const float* dxr, const float* dxl,
                             const float* dres, float* dacc, float* dWl, float* part, float* scratch, void* stream);
/* dh = dv Wm, dWm = dv^T h, dx = dv + LN_bwd(mask dh) (= d prev), dagg = dx Wp; partial rows. */
int gasfm_view_chain_tail_bwd(const float* dv, const float* x, const float* h, const float* rs, const float* agg,
                              int64_t m, int32_t D, const float* Wp, const float* ln_w, const float* ln_b,
                              const float* Wm, float* dh, float* dWm, float* dx, float* dagg, float* part,
                              float* scratch, uint32_t* counters, void* stream);

/* Batched single-row problems in ONE launch each way (the global hub: the LayerNorm -> Linear
 * consumers of a block's global row, then the two lin_r rows).  Arrays of nprob (<= 4) entries,
 * one per problem, as for gasfm_gvec_fwd / gasfm_gvec_bwd; null entries mean "absent" where the
 * single-problem calls accept null.  Backward: per-problem dW / db / dgamma / dbeta and partials
 * part[q] ([gasfm_gvec_bwd_chunks(N[q]) x K[q]]), then ngroups (<= 4) groups of problems that share
 * their input row: group g covers problems [g_p0[g], g_p0[g] + g_np[g]) and writes
 * dx[g] = dres[g] (may be null) + the sum of the group's backward terms. */
int gasfm_gvec_multi_fwd(int32_t nprob, const float* const* x, const float* const* ln_w, const float* const* ln_b,
                         const float* const* W, const float* const* b, const float* const* res, float* const* y,
                         const int32_t* K, const int32_t* N, float eps, void* stream);
int gasfm_gvec_multi_bwd(int32_t nprob, const float* const* dy, const float* const* x, const float* const* ln_w,
                         const float* const* ln_b, const float* const* W, const int32_t* K, const int32_t* N,
                         float* const* dW, float* const* db, float* const* dgam, float* const* dbet,
                         float* const* part, int32_t ngroups, const int32_t* g_p0, const int32_t* g_np,
                         const float* const* dres, float* const* dx, float eps, void* stream);

/* ---- calibrated camera head (baseNet.py:38-56, rot_representation 'quat') ----
 * P[c] = [R(q) | t] (3 x 4, row-major) from x[c] = (r, i, j, k, tx, ty, tz) (row stride ldx);
 * R is pytorch3d's quaternion_to_matrix (real part first, normalised by |q|^2).  Backward writes
 * dx[c] (7 values, row stride lddx). */
int gasfm_pose_fwd(const float* x, int64_t ldx, int64_t m, float* P, void* stream);
int gasfm_pose_bwd(const float* x, int64_t ldx, int64_t m, const float* dP, float* dx, int64_t lddx, void* stream);

/* ---- ESFMLoss over the visibility edges (esfm_loss.hip) ----
 * Replaces ESFMLoss.forward (code/loss_functions.py:85-123) and the gradient hook it registers
 * (loss_functions.py:104-113), which form the dense projections Ps @ pts3D [m, 3, n].  Per edge
 * e = (cam[e], pt[e]) with measurement vals[e] (= norm_M at that (camera, point)):
 * y = P[cam] @ pts3D[:, pt] (P: [m, 12] row-major 3x4, pts3D: [4, n] row-major).
 * Forward writes gasfm_esfm_part_rows(E) rows of (sum of loss terms, count of valid-depth
 * projections); their column sums are (E * loss, #pos).  Backward reads dloss[0] and
 * tot = (sum, #pos) from device memory and writes dP [m, 12] (cam_ptr: camera CSR over the
 * camera-sorted edges) and dpts3D [4, n] (pt_ptr + perm: point CSR, perm = edge ids in point
 * order, NULL = identity).  equalize / valid_only: pts_grad_equalization_pre_perspective_divide /
 * normalize_grad_wrt_valid_projections_only; hinge selects the hinge_loss branch
 * (geo_utils.get_positive_projected_pts_mask, geo_utils.py:721-726).  E_norm: the edge count the
 * mean divides by (E on one GPU; the GLOBAL count on a point-sharded scene, where each rank
 * passes its own edges: loss_functions.py:110 divides by the global sum(valid_pts)). */
int32_t gasfm_esfm_part_rows(int64_t E);
int gasfm_esfm_fwd(const int32_t* cam, const int32_t* pt, const float* vals, int64_t E, const float* P,
                   const float* pts3D, int64_t n, float margin, float hinge_w, int32_t hinge, float* part,
                   void* stream);
int gasfm_esfm_bwd(const int32_t* cam_ptr, int32_t m, const int32_t* pt_ptr, const int32_t* perm, const int32_t* cam,
                   const int32_t* pt, const float* vals, int64_t E, int64_t E_norm, const float* P,
                   const float* pts3D, int64_t n, float margin, float hinge_w, int32_t hinge, int32_t equalize,
                   int32_t valid_only, const float* dloss, const float* tot, float* dP, float* dpts3D, void* stream);

/* Union batch of S scenes in one edge list (the captured training step, gasfm_amd/static_batch.py):
 * scene s owns edges [eoff[s], eoff[s+1]) and the cameras / points scene_of_cam / scene_of_pt map
 * to s.  Forward: tot[s] = (sum of loss terms, #pos) of scene s, loss[0] = sum over the scenes with
 * weight[s] != 0 of weight[s] * tot[s][0] / E_s (train.py:76-96 sums the per-scene ESFMLoss of a
 * batch); part: gasfm_esfm_seg_part_rows(S) x 2 floats of workspace.  Backward: each camera's /
 * point's gradient as gasfm_esfm_bwd with that scene's E_s and tot[s], scaled by weight[s]; a
 * scene of weight 0 (padding) gets exact zeros.  S <= 256.  Fixed launch geometry for a given S,
 * so the calls replay inside a captured graph while the edge counts in eoff change. */
int32_t gasfm_esfm_seg_part_rows(int32_t S);
int gasfm_esfm_seg_fwd(const int32_t* cam, const int32_t* pt, const float* vals, const int32_t* eoff, int32_t S,
                       const float* weight, const float* P, const float* pts3D, int64_t n, float margin,
                       float hinge_w, int32_t hinge, float* part, float* tot, float* loss, void* stream);
int gasfm_esfm_seg_bwd(const int32_t* cam_ptr, int32_t m, const int32_t* pt_ptr, const int32_t* perm,
                       const int32_t* cam, const int32_t* pt, const float* vals, const int32_t* eoff, int32_t S,
                       const int32_t* scene_of_cam, const int32_t* scene_of_pt, const float* weight, const float* P,
                       const float* pts3D, int64_t n, float margin, float hinge_w, int32_t hinge, int32_t equalize,
                       int32_t valid_only, const float* dloss, const float* tot, float* dP, float* dpts3D,
                       void* stream);

/* ---- global node (ONE row): LayerNorm -> ReLU -> Linear (+ residual) ----
 * Replaces the M = 1 aten chains on the global feature vector: norm_and_proj_global2view /
 * _global2scenepoint (layers.py:497-520), both convs' lin_r on those rows (PyG),
 * proj_view_and_scenepoint2global + g (layers.py:527-528, 590-592), the pre-MLP skip
 * (layers.py:594-603) and lin_global of the projection update (layers.py:928-935).
 * K (input width) must be a multiple of 64 and <= 4096. */

/* y[i] = W[i,:] . h + b[i] (+ res[i]), h = relu(LN(x)) if ln_w else x.  x: [K], W: [N x K]
 * row-major, b / res may be null. */
int gasfm_gvec_fwd(const float* x, int32_t K, const float* ln_w, const float* ln_b, float eps,
                   const float* W, const float* b, int32_t N, const float* res, float* y, void* stream);

/* Rows of the partial buffer gasfm_gvec_bwd needs: part is [gasfm_gvec_bwd_chunks(N) x K]. */
int gasfm_gvec_bwd_chunks(int32_t N);

/* Backward of the above: dW = dy (x) h, db = dy (db may be null), dx = LN_bwd(mask * W^T dy)
 * (+ dy when resid, i.e. the residual was x itself; needs N == K), dgamma, dbeta.  Two
 * launches (slab pass + one-workgroup finish), deterministic. */
int gasfm_gvec_bwd(const float* dy, const float* x, int32_t K, const float* ln_w, const float* ln_b,
                   float eps, const float* W, int32_t N, int32_t resid, float* dx, float* dW, float* db,
                   float* dgamma, float* dbeta, float* part, void* stream);

/* ---- the global node's whole chain of one block (global_chain.hip, round 4) ----
 * Replaces, as ONE forward / backward pair of four launches each, the per-block single-row chain
 * ViewAndScenePoint2Global's tail (layers.py:527-528, 590-603: x1 = W1 xcat + b1 (+ prev),
 * g = x1 + W2 relu(LN_M(x1)) + b2) and every consumer of g: lin_global of the projection update
 * (layers.py:928-935: SG = WA relu(LN_A(g))), the next block's norm_and_proj_global2view /
 * _global2scenepoint (layers.py:497-520: xv = WB relu(LN_B(g)) + bWB, xp = WC relu(LN_C(g)) + bWC)
 * and the two lin_r rows of the next block's global GATv2 convs (PyG: XRv = WD xv + bD,
 * XRp = WE xp + bE).  NB = 0 (and NC = ND = NE = 0): the last block, whose g has SG only.
 * Widths G, Kc, NB, NC: multiples of 32, <= 2048.  All weights row-major [out, in], 16-byte aligned. */
typedef struct gasfm_gchain {
  int32_t G, Kc, NA, NB, NC, ND, NE;
  float eps_m, eps_h; /* norm_pre_mlp eps; the hub LayerNorms' (shared) eps */
  const float *W1, *b1, *gM, *bM, *W2, *b2;
  const float *gA, *bA, *WA;
  const float *gB, *bB, *WB, *bWB, *gC, *bC, *WC, *bWC;
  const float *WD, *bD, *WE, *bE;
  /* optional bf16 shadows (round 5, BASELINE config 5: the weights rounded to bf16, refreshed by the
   * caller once per optimizer step; NULL: read the fp32 weight).  The GEMVs stream half the weight
   * bytes and accumulate in fp32; every gradient stays fp32 (dW = dy x h does not read W). */
  const uint16_t *W1h, *W2h, *WAh, *WBh, *WCh, *WDh, *WEh;
  /* rows (round 5): the chain on `rows` global rows at once -- a union batch's one global node per
   * scene (train.py's batch as one forward; gasfm_amd/static_batch.py), every weight streamed once
   * for all of them.  0 or 1: one row.  Every activation / gradient vector argument of
   * gasfm_gchain_fwd / _bwd is then [rows, len] row-major; the parameter gradients sum the rows.
   * rows <= GASFM_GCHAIN_MAX_ROWS. */
  int32_t rows;
} gasfm_gchain;
#define GASFM_GCHAIN_MAX_ROWS 7
typedef struct gasfm_gchain_grads {
  float *dW1, *db1, *dgM, *dbM, *dW2, *db2;
  float *dgA, *dbA, *dWA;
  float *dgB, *dbB, *dWB, *dbWB, *dgC, *dbC, *dWC, *dbWC;
  float *dWD, *dbD, *dWE, *dbE;
} gasfm_gchain_grads;

/* Forward: xcat [Kc], prev [G] or NULL -> x1, g [G], sg [NA] (and xv [NB], xp [NC], xrv [ND],
 * xrp [NE] when NB > 0). */
int gasfm_gchain_fwd(const gasfm_gchain* c, const float* xcat, const float* prev, float* x1, float* g, float* sg,
                     float* xv, float* xp, float* xrv, float* xrp, void* stream);
/* Scratch floats and ticket counters (zeroed, self-resetting) gasfm_gchain_bwd needs. */
int64_t gasfm_gchain_scratch_floats(const gasfm_gchain* c);
int32_t gasfm_gchain_counters(const gasfm_gchain* c);
/* Backward from d g (dskip, may be NULL), d SG, d XRv, d XRp -> d xcat [Kc], d prev [G] (may be
 * NULL when the forward had no prev) and every parameter gradient (grads of absent hub terms
 * ignored).  Deterministic (no float atomics). */
int gasfm_gchain_bwd(const gasfm_gchain* c, const float* xcat, const float* x1, const float* g, const float* xv,
                     const float* xp, const float* dskip, const float* dsg, const float* dxrv, const float* dxrp,
                     float* dxcat, float* dprev, const gasfm_gchain_grads* d, float* scratch, uint32_t* counters,
                     void* stream);

/* ---- the two GATv2 convs onto the single global node (global_attn.hip, round 4) ----
 * graph_conv_view2global / graph_conv_scenepoint2global (layers.py:550-556, 566-572; PyG GATv2Conv,
 * H = 4 heads, one target): e_j = att . leaky(XL[src_j] + XR), alpha = softmax_j(e_j) per head,
 * out = sum_j alpha_j XL[src_j] + bias.  Up to two problems (views C = 256, points C = 16) per
 * launch.  src NULL = rows 0..S-1.  Forward writes out [HC] and the statistics smax / ssum [H]
 * (the softmax max and sum), or, when part != NULL (a sharded rank), the packed partial row
 * [acc HC | max H | sum H] instead.  Backward (from gout, the saved out / smax / ssum) writes the
 * dXL rows of the S sources (other rows untouched), dXR [HC] and datt [2 HC] = datt | dbias
 * (dbias = gout).  S = 0 is allowed (a rank without sources: the empty state / zero gradients).
 * XL, XR, att, bias, out, gout, dXL, datt 16-byte aligned; ldXL, ldDXL multiples of 4. */
typedef struct gasfm_gatt_prob {
  const float* XL;
  int64_t ldXL;
  const int32_t* src;
  int32_t S, HC;
  const float *XR, *att, *bias;
  float *out, *smax, *ssum, *part;
  const float* gout;
  float* dXL;
  int64_t ldDXL;
  float *dXR, *datt;
} gasfm_gatt_prob;
int64_t gasfm_gatt_scratch_floats(int32_t nprob, const gasfm_gatt_prob* probs);
/* counters: gasfm_gatt_counters(nprob, probs) zeroed self-resetting tickets (one per problem, plus
 * one per group of 32 source chunks when a problem has more than 32 chunks: two-level merge). */
int32_t gasfm_gatt_counters(int32_t nprob, const gasfm_gatt_prob* probs);
int gasfm_gatt_fwd(int32_t nprob, const gasfm_gatt_prob* probs, float slope, float* scratch, uint32_t* counters,
                   void* stream);
int gasfm_gatt_bwd(int32_t nprob, const gasfm_gatt_prob* probs, float slope, float* scratch, uint32_t* counters,
                   void* stream);
/* The sharded forward's merge of the gathered partial rows: problem q's row of rank r at
 * probs[q].part + r * stride floats (r < nrows), merged (max, rescaled sums) into out / smax / ssum
 * (+ bias), the same on every rank.  One workgroup per problem, one launch. */
int gasfm_gatt_merge(int32_t nprob, const gasfm_gatt_prob* probs, int32_t nrows, int64_t stride, void* stream);

/* The camera-sharded block exchange (round 5): one all-gather of per-rank send blocks carries
 * several payloads.  G holds W send blocks of blk floats; rank r's block carries at float offset
 * roff its chunk own rows of width floats (rows past the scene's m are padding) and at soff a
 * partial vector of sn floats.  rows_dst [m, width] (row stride ld_dst; may be null) receives camera
 * row c = G[(c / chunk) blk + roff + (c % chunk) width ..]; sum_dst [sn] (may be null) the W
 * partial vectors summed in rank order (the same bits on every rank).  blk, roff, soff, width,
 * ld_dst, sn multiples of 4; 16-byte aligned pointers.  Replaces (reference: none, the reference
 * is single-device) a second collective per block: the forward's view-row gather rides with the
 * global convs' partial rows, the backward's camera-aggregate gradient gather with the global
 * target rows' gradient sum. */
int gasfm_exchange_unpack(const float* G, int32_t W, int64_t blk, int64_t roff, int32_t chunk, int32_t width,
                          int32_t m, float* rows_dst, int64_t ld_dst, int64_t soff, int32_t sn, float* sum_dst,
                          void* stream);
/* gasfm_gatt_merge and gasfm_exchange_unpack's row copy (no sum) in ONE launch. */
int gasfm_gatt_merge_unpack(int32_t nprob, const gasfm_gatt_prob* probs, int32_t nrows, int64_t stride,
                            const float* G, int32_t W, int64_t blk, int64_t roff, int32_t chunk, int32_t width,
                            int32_t m, float* rows_dst, int64_t ld_dst, void* stream);

/* Reprojection error of compute_core_errors' "our_repro" (code/evaluation.py:8-31 ->
 * geo_utils.reprojection_error_with_points, geo_utils.py:371-391) over the E visibility edges:
 * err_e = || xy_e - (P_c X)_xy / (P_c X)_z ||, X = pflat(pts3D[:, p]), P = Ps_pix [m x 12]
 * (= Ns^-1 Ps_norm), xy = PIXEL measurements [E x 2].  err (optional, [E]) per edge;
 * part [gasfm_esfm_part_rows(E) x 2] = per-workgroup (sum of non-NaN errors, their count), the
 * operands of np.nanmean (finish with gasfm_colsum). */
int gasfm_reproj_error(const int32_t* cam, const int32_t* pt, const float* xy, int64_t E, const float* P,
                       const float* pts3D, int64_t n, float* err, float* part, void* stream);
/* ---- Adam over all parameter tensors in one launch (adam.hip; gasfm_amd/optim.py) ----
 * torch.optim.Adam's update (amsgrad off, maximize off; torch/optim/adam.py) for every tensor of
 * the table at optimizer step `step` (>= 1): g' = g + weight_decay p, m += (1 - beta1)(g' - m),
 * v = beta2 v + (1 - beta2) g'^2, p -= lr / (1 - beta1^step) m / (sqrt(v) / sqrt(1 - beta2^step)
 * + eps).  chunks: one entry per GASFM_ADAM_CHUNK values of a tensor (tensor index, first value),
 * one workgroup each.  p / m / v are updated in place; g is read. */
#define GASFM_ADAM_CHUNK 4096
typedef struct gasfm_adam_tensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t numel;
} gasfm_adam_tensor;
typedef struct gasfm_adam_chunk {
  int32_t tensor;
  int32_t reserved;
  int64_t begin;
} gasfm_adam_chunk;
int gasfm_adam_step(const gasfm_adam_tensor* tensors, const gasfm_adam_chunk* chunks, int32_t n_chunks, double lr,
                    double beta1, double beta2, double eps, double weight_decay, int64_t step, void* stream);

/* ---- a union batch's per-scene global term folded into its cameras' rows (static_batch.hip) ----
 * model._fold_global (batch.py's union of scenes, one global node per scene): forward
 * out[c] = sv[c] + sg[soc[c]] ([m x width] rows, row strides given); backward dsg[s] = the sum over
 * the cameras of scene s of dout[c], in camera order (one workgroup per scene, no atomics). */
int gasfm_fold_scene_rows_fwd(const float* sv, int64_t ldsv, const float* sg, int64_t ldsg, const int64_t* soc,
                              int64_t m, int32_t width, float* out, int64_t ldo, void* stream);
int gasfm_fold_scene_rows_bwd(const float* dout, int64_t ld, const int64_t* soc, int64_t m, int32_t S,
                              int32_t width, float* dsg, int64_t ldsg, void* stream);

/* ---- shape-stable union batch fill (static_batch.hip; gasfm_amd/static_batch.py) ----
 * The captured config-3 / config-5 training step (train.py:60-152) replays one graph per bucket of
 * fixed cameras / points / edges / camera items; each step writes the sampled scenes and a pad
 * scene into the bucket's static buffers.  gasfm_union_fill_scene writes scene s at union offsets
 * (e0, c0, p0): indices [2 x E_cap] (row stride ld_indices) and their int32 copies, the network's
 * and the loss's measurements, pixel measurements gathered from the scene's dense M [2m x n] (row
 * stride ldM; NULL: zeros), perm / pos (point-order edge ids and their inverse; NULL: identity) and
 * both CSRs offset by e0, cam_per_pts / pts_per_cam, the scene maps, Ns^-1 per camera (fp64
 * inverse, fp32 out), one point work item per point (slot -1) and ceil(deg / piece) camera work
 * items per camera from item0 on, every camera through partial slots (slot = item index) with one
 * combine entry (c, first, pieces, 1).  m <= GASFM_UNION_MAX_CAMS.  gasfm_union_fill_pad writes
 * the pad scene after the real ones: mp cameras / npd points / ep edges from (M, N, E), degrees
 * spread evenly, edge k joining the k-th entries of the two degree expansions, zero measurements,
 * identity Ns^-1, the remaining dI camera items from item0 on, and the closing CSR entries. */
#define GASFM_UNION_MAX_CAMS 4096
typedef struct gasfm_union_scene {
  const int64_t* idx; /* [2 x E] (cam, pt), row stride ld_idx */
  int64_t ld_idx;
  const float* vals;      /* [E x 2] the network's measurements */
  const float* vals_loss; /* [E x 2] the loss's (the clean scene under outlier injection) */
  const int32_t* cptr;    /* [m + 1] */
  const int32_t* pptr;    /* [n + 1] */
  const int32_t* perm;    /* [E] or NULL */
  const int32_t* pos;     /* [E] or NULL */
  const int64_t* cam_per_pts; /* [n] */
  const int64_t* pts_per_cam; /* [m] */
  const float* M;             /* [2m x n] or NULL */
  int64_t ldM;
  const float* Ns; /* [m x 3 x 3] */
  int64_t E, m, n;
  int64_t e0, c0, p0, item0;
  int32_t scene;
} gasfm_union_scene;
typedef struct gasfm_union_out {
  int64_t* indices;
  int64_t ld_indices;
  int32_t *cam32, *pt32;
  float *values, *values_loss, *xy;
  int32_t *perm, *pos, *cam_ptr, *pt_ptr;
  int64_t *cam_per_pts, *pts_per_cam, *soc;
  int32_t *soc32, *sop32;
  float* Ns_inv;
  int32_t *items_c, *comb_c, *items_p;
  int32_t piece;
} gasfm_union_out;
typedef struct gasfm_union_pad {
  int64_t M, N, E, mp, npd, ep, dI, item0;
  int32_t scene;
} gasfm_union_pad;
int gasfm_union_fill_scene(const gasfm_union_scene* scene, const gasfm_union_out* out, void* stream);
int gasfm_union_fill_pad(const gasfm_union_pad* pad, const gasfm_union_out* out, void* stream);

/* The same per scene of a union batch (eoff, S as gasfm_esfm_seg_fwd): tot[s] = (sum of the
 * non-NaN errors of scene s, their count); part: gasfm_esfm_seg_part_rows(S) x 2 floats. */
int gasfm_reproj_error_seg(const int32_t* cam, const int32_t* pt, const float* xy, const int32_t* eoff, int32_t S,
                           const float* P, const float* pts3D, int64_t n, float* part, float* tot, void* stream);

/* ---- device-side scene graph builder (scene_build.hip) ------------------
 * For a dense measurement matrix M [2m x n] (row stride ldM floats) already in HBM, builds on
 * the device what the reference builds on the CPU per sample:
 *   get_M_valid_points (dataset_utils.py:86-113), M2sparse + normalize_M (dataset_utils.py:116-156,
 *   geo_utils.py:689-703), and the stable point-direction grouping of gasfm_build_csr.
 * Workspace: mask [m x gasfm_scene_mask_words(n)] uint64 (one bit per camera/point),
 * pt_valid [gasfm_scene_mask_words(n)] uint64, view_count / pt_count [n], tile_count
 * [gasfm_scene_tiles(m, n)], tile_base [gasfm_scene_tiles(m, n) + 1], word_base [m x words].
 * Requires m*n < 2^31 (int32 edge ids).  Deterministic (integer atomics only). */
int64_t gasfm_scene_mask_words(int32_t n);
int64_t gasfm_scene_tiles(int32_t m, int32_t n);

/* Exclusive scan: out[0..L) = prefix sums of in, out[L] = total (int32).  One workgroup. */
int gasfm_scan_i32(const int32_t* in, int64_t L, int32_t* out, void* stream);

/* Pass 1: validity bits ((x, y) != (0, 0)), raw views per point (view_count), points with
 * >= 2 views (pt_valid bits; pt_count = view_count or 0 = the reference's cam_per_pts), and
 * the per-tile edge counts with their exclusive scan: E = tile_base[tiles]. */
int gasfm_scene_mask(const float* M, int64_t ldM, int32_t m, int32_t n, uint64_t* mask,
                     int32_t* view_count, uint64_t* pt_valid, int32_t* pt_count, int32_t* tile_count,
                     int32_t* tile_base, void* stream);

/* Pass 2: the E edges in the reference's nonzero() order (cam-major, point ascending):
 * cam[E], pt[E] (int64, the reference's SparseMat.indices rows) and values [E x 2]
 * (N_c [x, y, 1]^T rows 0..1 when Ns [m x 3 x 3] != NULL, raw (x, y) otherwise), plus
 * word_base (edge id of the first edge of each mask word) for pass 3. */
int gasfm_scene_emit(const float* M, int64_t ldM, const float* Ns, int32_t m, int32_t n,
                     const uint64_t* mask, const uint64_t* pt_valid, const int32_t* tile_base,
                     int64_t* cam, int64_t* pt, float* values, int32_t* word_base, void* stream);

/* Pass 3: point-direction CSR given pt_ptr = exclusive scan of pt_count: perm[slot] = edge
 * (stable, cameras ascending inside a point; == gasfm_build_csr on pt) and pos[edge] = slot. */
int gasfm_scene_point_csr(const uint64_t* mask, const uint64_t* pt_valid, const int32_t* word_base,
                          const int32_t* pt_ptr, int32_t m, int32_t n, int32_t* perm, int32_t* pos,
                          void* stream);

/* Rotational homography augmentation of the image points (SceneData.apply_rotational_homography_aug,
 * datasets/SceneData.py:355-440): out[2c:2c+2, p] = pflat(Ninv_c R_c Ns_c [x, y, 1]^T)[:2] where
 * (c, p) is valid (mask / pt_valid from gasfm_scene_mask on M), 0 elsewhere.  Ns, R, Ninv:
 * [m x 3 x 3] row-major; out may not alias M. */
int gasfm_scene_homography(const float* M, int64_t ldM, int32_t m, int32_t n, const uint64_t* mask,
                           const uint64_t* pt_valid, const float* Ns, const float* R, const float* Ninv,
                           float* out, int64_t ldO, void* stream);

/* dst[i] = src[0][i] + ... + src[n-1][i] (index order), n <= 16, count % 4 == 0, 16-byte aligned
 * rows: the gradient of a tensor with n consumers in one pass (the embedded projection input P0
 * feeds every block's projection update, layers.py:245-251; autograd would add n-1 times). */
int gasfm_sum_n(int32_t n, const float* const* src, int64_t count, float* dst, void* stream);

/* bf16 MFMA GEMM with fp32 operands and result (BASELINE config 5's "bf16 projections on MFMA";
 * replaces the m x 1024 x 1024 Linear products of Proj2View's MLP and graph_conv_view2global.lin_l,
 * code/models/layers.py:292-320, 352-358, 506-511, forward and both backward products):
 *   C[M,N] = A[M,K] . B[K,N] (+ Cin[M,N]) (+ bias[N]),  A(i,k) = A[i*sAm + k*sAk],
 *   B(k,j) = B[k*sBk + j*sBn].  Operands are rounded to bf16 (nearest even) on the way into LDS,
 * multiplied exactly and accumulated in fp32.  One of sAm / sAk and one of sBk / sBn must be 1;
 * the extent along the unit stride and the other stride are multiples of 4, A and B 16-byte
 * aligned.  C may alias Cin (same ld); it may not alias A or B. */
int gasfm_gemm_bf16(int32_t M, int32_t N, int32_t K, const float* A, int64_t sAm, int64_t sAk,
                    const float* B, int64_t sBk, int64_t sBn, const float* Cin, int64_t ldCin,
                    const float* bias, float* C, int64_t ldC, void* stream);

/* The same product in fp32 on v_mfma_f32_16x16x4_f32 (exact products, fixed-order fp32 sums):
 * the camera-side D x D Linear layers at m = 1000 (one GPU) and m = 125 (a camera shard of 8).
 * Replaces torch.addmm / mm (hipBLASLt) at layers.py:292-320, 352-358, 506-511. C may equal Cin. */
int gasfm_gemm_f32(int32_t M, int32_t N, int32_t K, const float* A, int64_t sAm, int64_t sAk,
                   const float* B, int64_t sBk, int64_t sBn, const float* Cin, int64_t ldCin,
                   const float* bias, float* C, int64_t ldC, void* stream);

/* fp32 MFMA GEMMs for small row counts (gemm_smallm.hip: a camera-sharded rank's m / W view rows):
 *   mode 0  C[M,N] = A[M,K] W[N,K]^T (+ bias[N]) (+ Cin[M,N]); A, W row-major (lda, ldb)
 *   mode 1  C[M,N] = A[M,K] W[K,N]; bias / Cin must be null
 *   mode 2  C[M,N] = A[K,M]^T B[K,N] (K: rows, any); bias / Cin must be null
 * gasfm_gemm_f32_smallm_ok says whether (mode, M, N, K) is supported (modes 0 / 1: K % 64 == 0,
 * N % 32 == 0; mode 2: M % 16 == 0, N % 128 == 0).  Cin may alias C. */
int32_t gasfm_gemm_f32_smallm_ok(int32_t mode, int32_t M, int32_t N, int32_t K);
int gasfm_gemm_f32_smallm(int32_t mode, int32_t M, int32_t N, int32_t K, const float* A, int64_t lda, const float* B,
                          int64_t ldb, const float* bias, const float* Cin, int64_t ldCin, float* C, int64_t ldC,
                          void* stream);

/* ---- outlier injection (outliers.hip) -----------------------------------
 * Replaces OutlierInjector / inject_outliers (code/utils/dataset_utils.py:159-461), the per-sample
 * transform of the outlier-injected training loop (train.py:73-81, BASELINE config 5).  The
 * partition of the E projections (camera-major M2sparse order) is one byte per edge:
 * 0 fixed inlier, 1 fixed outlier, 2 free inlier, 3 free outlier (bit 0 = outlier).  The random
 * choices between the passes are the caller's (the reference's numpy draws). */

/* Inliers per view (cam_in [m], segments cam_ptr [m+1]) and per point (pt_in [n], CSR pt_ptr
 * [n+1] with perm slot -> edge, NULL = identity); mins[0] / mins[1] = their minima. */
int gasfm_outlier_counts(const uint8_t* state, const int32_t* cam_ptr, const int32_t* pt_ptr,
                         const int32_t* perm, int32_t m, int32_t n, int32_t* cam_in, int32_t* pt_in,
                         int32_t* mins, void* stream);

/* mode 0 (init_fixed_inliers_and_outliers, :253-275): state = 0 where pt_in[pt] < 3 or
 * cam_in[cam] < 9, else 2 (cam_in / pt_in = all projections).  mode 1
 * (blacklist_problematic_outliers, :307-320): a free outlier whose point has < 2 or whose view
 * has < 8 remaining inliers (cam_in / pt_in from gasfm_outlier_counts) becomes 0.
 * counts[0..3] = edges per class afterwards. */
int gasfm_outlier_mark(uint8_t* state, const int64_t* cam, const int64_t* pt, const int32_t* cam_in,
                       const int32_t* pt_in, int64_t E, int32_t mode, int32_t* counts, void* stream);

/* Per view over the inliers of the pixel values [E x 2] (sparse_moment_estimation,
 * sparse_utils.py:151-165): mu [m x 2], sigma [m x 2 x 2] = sum x x^T / (N - 1), and
 * scale_tril [m x 2 x 2] with sigma = T T^T from the LDL^T factorisation of LAPACK sytf2
 * (lower, Bunch-Kaufman; pivots [m x 2] as torch.linalg.ldl_factor reports them, negative =
 * 2x2 block, then scale_tril is NaN) with the reference's row flip (:378-392). */
int gasfm_outlier_moments(const float* values, const uint8_t* state, const int32_t* cam_ptr, int32_t m,
                          float* mu, float* sigma, float* scale_tril, int32_t* pivots, void* stream);

/* Outlier k (edge idx[k], ascending): value = mu[cam] + scale_tril[cam] z[k] (z [n_out x 2]),
 * written into the dense pixel matrix M [2m x ldM] and, if pix != NULL, pix [E x 2] (:397-433). */
int gasfm_outlier_apply(const int64_t* idx, int64_t n_out, const int64_t* cam, const int64_t* pt,
                        const float* z, const float* mu, const float* scale_tril, float* M, int64_t ldM,
                        float* pix, void* stream);

/* ---- bundle adjustment (bundle_adjust.hip) --------------------------------
 * The reference's Ceres problem (bundle_adjustment/custom_cpp_cost_functions.cpp:56-222; driven by
 * code/utils/ba_functions.py:6-137 / ceres_utils.py:127-245) as device passes of a trust-region
 * Levenberg-Marquardt with the points eliminated (DENSE_SCHUR), fp64.  cp = 6: Euclidean camera
 * deltas (angle-axis, t) with cam0 [m x 6] and K [m x 5] (K00 K01 K02 K11 K12); cp = 12:
 * projective P deltas (column-major 3 x 4), K unused.  Edges are camera-major (cam_ptr [m+1]);
 * the point CSR (pt_ptr [n+1], perm slot -> edge, NULL = identity) lists cameras ascending.
 * Huber(0.1) enters through Ceres' corrector (residual and Jacobian scaled by sqrt(rho')). */
int64_t gasfm_ba_partials(int64_t E);  /* per-workgroup partial count of eval / model */

/* cost partials (1/2 rho per edge, summed per workgroup) at (cam0 + dcam, X0 + dX); with jac:
 * corrected residuals fres [E x 2] and Jacobians Jc [E x 2 x cp], Jp [E x 2 x 3], columns
 * scaled by sc [m x cp] / sp [n x 3] (NULL = 1). */
int gasfm_ba_eval(int32_t cp, const double* cam0, const double* K, const double* X0, const double* dcam,
                  const double* dX, const int32_t* cidx, const int32_t* pidx, const double* obs, int64_t E,
                  const double* sc, const double* sp, int32_t jac, double* fres, double* Jc, double* Jp,
                  double* part, void* stream);
/* out[0] = sum of part[0..count) in a fixed order (one workgroup). */
int gasfm_ba_sum(const double* part, int64_t count, double* out, void* stream);
/* U [m x cp x cp] = Jc^T Jc and gc [m x cp] = Jc^T f per camera; V [n x 3 x 3], gp [n x 3] per point. */
int gasfm_ba_normals(int32_t cp, int32_t m, int32_t n, const int32_t* cam_ptr, const int32_t* pt_ptr,
                     const int32_t* perm, const double* fres, const double* Jc, const double* Jp, double* U,
                     double* gc, double* V, double* gp, void* stream);
/* LM damping: Ud = U + clamp(diag U, 1e-6, 1e32) / radius; Vinv = (V + same)^-1; *bad = 1 if a point
 * block is not positive definite (the caller zeroes *bad). */
int gasfm_ba_damp(int32_t cp, int32_t m, int32_t n, const double* U, const double* V, double radius,
                  double* Ud, double* Vinv, int32_t* bad, void* stream);
/* Reduced camera system: Y [E x cp x 3] workspace, S [(m cp) x (m cp)] dense row-major, rhs [m cp].
 * Camera-pair blocks (a <= b) blk_ab [nblk x 2] with pair ranges blk_ptr [nblk+1] into the edge
 * pairs (pe1 [P] on camera a, pe2 [P] on camera b, same point). */
int gasfm_ba_schur(int32_t cp, int32_t m, const int32_t* cam_ptr, const int32_t* cidx, const int32_t* pidx,
                   int64_t E, const double* Jc, const double* Jp, const double* Vinv, const double* gc,
                   const double* gp, const double* Ud, const int32_t* blk_ptr, const int32_t* blk_ab,
                   int64_t nblk, const int32_t* pe1, const int32_t* pe2, double* Y, double* S, double* rhs,
                   void* stream);
/* dp [n x 3] = Vinv (-gp - sum_e W_e^T dc[cam]) for the camera step dc [m x cp]. */
int gasfm_ba_backsub(int32_t cp, int32_t n, const int32_t* pt_ptr, const int32_t* perm, const int32_t* cidx,
                     const double* Jc, const double* Jp, const double* Vinv, const double* gp, const double* dc,
                     double* dp, void* stream);
/* model cost change partials: -(mr . (f + mr / 2)), mr = Jc dc + Jp dp, per workgroup. */
int gasfm_ba_model(int32_t cp, const int32_t* cidx, const int32_t* pidx, int64_t E, const double* Jc,
                   const double* Jp, const double* fres, const double* dc, const double* dp, double* part,
                   void* stream);
/* DLT triangulation (geo_utils.dlt_triangulation, code/utils/geo_utils.py:611-656): X [n x 4],
 * X[3] = 1, NaN for points in < 2 views; nP [m x 3 x 4] normalised cameras, nx [E x 2]
 * normalised observations. */
int gasfm_ba_dlt(int32_t n, const int32_t* pt_ptr, const int32_t* perm, const int32_t* cidx, const double* nP,
                 const double* nx, double* X, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GASFM_H */
