// Generic NHWC layer kernels (ops_generic.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace gops {

struct ConvShape {
  int N, H, W, C;  // input
  int K;           // output channels
  int R, S;        // kernel
  int stride, pad;
  int OH, OW;
};

struct PoolShape {
  int N, H, W, C, k, stride, pad, OH, OW;
};

// ws: split-K workspace of conv_ws_floats(s, bias || relu) floats (shared by
// the three ops of one layer; dw / dx / y are written, not accumulated)
// bf16: MFMA operands converted to bf16 (fp32 accumulate, fp32 in / out); the
// tiled family only - shapes it does not take run the fp32 gather engine
// xb / dyb: optional bf16 copies of x / dy (to_bf16) for the bf16 family
// wtb (optional, bf16 family): the weights already laid out by wcvt_batch
// (forward copy for conv_fwd, stride-1 dgrad copy for conv_bwd_data)
// yb (optional, bf16 family only): write the output as bf16 there instead of y
// BatchNorm statistics from a bf16-output conv (the bf16 family's epilogue,
// or its split-K reduction): partial sums of (y - shift[c]) and
// (y - shift[c])^2 over the output rows, part [2][K / 64][P][64] with P =
// conv_fwd_stats_rows(s) (y = the bf16-rounded outputs the BatchNorm reads;
// shift = the BatchNorm's running mean).  Consumed by bn_fwd_partials.
struct ConvStats {
  float* part = nullptr;
  int P = 0;
  const float* shift = nullptr;
};
// BatchNorm BACKWARD statistics from the dgrad that produces the BatchNorm's
// dY (bf16 family, fp32 dX): with d = dX [y > 0] (relu) and xhat = (x - mean)
// rstd, partial sums of d and d xhat over the rows, part [2][C / 64][P][64]
// with P = conv_bwd_data_stats_rows(s) (0: this dgrad cannot write them).  x =
// the BatchNorm's bf16 input, y = the bf16 twin of its output (ReLU mask).
// Consumed by bn_bwd_partials.
struct BnBwdStats {
  float* part = nullptr;
  int P = 0;
  const void* x = nullptr;  // bf16
  const void* y = nullptr;  // bf16 (relu only)
  const float* mean = nullptr;
  const float* rstd = nullptr;
  int relu = 0;
};
int conv_bwd_data_stats_rows(const ConvShape& s);
// bf16 = true: bf16 family, bf16 output; false: the fp32 tiled forward (no bias / ReLU)
int conv_fwd_stats_rows(const ConvShape& s, bool bf16 = true);
int conv_fwd_stem_stats_rows(const ConvShape& s1);
void conv_fwd(const ConvShape& s, const float* x, const float* w, const float* bias, float* y,
              bool relu, float* ws, hipStream_t st, bool bf16 = false, const void* xb = nullptr,
              const void* wtb = nullptr, void* yb = nullptr, const ConvStats* stats = nullptr);
// addend (optional, bf16 / tiled families): a gradient that joins dX at this
// tensor (a residual branch), added in the epilogue: dx = conv + addend
void conv_bwd_data(const ConvShape& s, const float* dy, const float* w, float* dx, float* ws,
                   hipStream_t st, bool bf16 = false, const void* dyb = nullptr,
                   const float* addend = nullptr, const void* wtb = nullptr,
                   const BnBwdStats* bstats = nullptr);
bool conv_bwd_data_join_ok(const ConvShape& s, bool bf16);  // takes an addend
int conv_filter_splits(const ConvShape& s);
void conv_bwd_filter(const ConvShape& s, const float* x, const float* dy, float* ws, float* dw,
                     hipStream_t st, bool bf16 = false, const void* xb = nullptr,
                     const void* dyb = nullptr);
long long conv_ws_floats(const ConvShape& s, bool fwd_epilogue);
// bf16 MFMA convs with 64-channel K tiles and pre-laid-out bf16 weights
// (conv_bf16.hip): forward for C, K % 64 == 0, stride-1 backward-data; the
// bf16 weight copy and split-K slabs live in the layer workspace
bool conv_fwd_bf16_ok(const ConvShape& s);
bool conv_bwd_data_bf16_ok(const ConvShape& s);
long long conv_bf16_ws_floats(const ConvShape& s, bool fwd_epilogue);
void to_bf16(const float* x, void* y, long long n, hipStream_t st);
void im2col_bf16(const ConvShape& s, const float* x, int kp, void* col, hipStream_t st);
// the stem conv over its implicit im2col (no column matrix): s1 = the 1x1
// GEMM shape over kp channels, si = the image conv, x = fp32 NHWC image,
// wtb = stem_weight_bf16 layout; yb = bf16 output; dw = padded [kp][K] grad
void conv_fwd_stem_bf16(const ConvShape& s1, const ConvShape& si, const float* x, const void* wtb,
                        void* yb, hipStream_t st, const ConvStats* stats = nullptr);
void conv_bwd_filter_stem_bf16(const ConvShape& s1, const ConvShape& si, const float* x,
                               const void* dyb, float* ws, float* dw, hipStream_t st);
// The ResNet stem (7x7 / stride 2 / pad 3 over 3 channels) by space-to-depth:
// a 4x4 / stride-1 conv over the bf16 s2d image xs [N][OH + 3][OW + 3][16]
// (s2d_stem_input) with the 8x8-extended filter wt8 [K][256] (s2d_stem_weight);
// si = ConvShape(N, OH + 3, OW + 3, 16, K, 4, 4, 1, 0).  Forward: bf16 output
// yb (+ BatchNorm statistics, conv_fwd_stem_stats_rows of the GEMM view);
// filter gradient: dw8 [256][K] fp32 (s2d_stem_wgrad maps it back to HWIO),
// ws of s2d_stem_ws_floats(si) floats.
void conv_fwd_s2d_stem_bf16(const ConvShape& si, const void* xs, const void* wt8, void* yb,
                            hipStream_t st, const ConvStats* stats);
// A/B: the s2d stem forward with every K tile requested at once (default) or
// one tile ahead (fwd_kernel's generic pipeline)
void s2d_stem_set_preload(bool on);
void conv_bwd_filter_s2d_stem_bf16(const ConvShape& si, const void* xs, const void* dyb,
                                   float* ws, float* dw8, hipStream_t st);
size_t s2d_stem_ws_floats(const ConvShape& si);
// x fp32 NHWC [N][H][W][3] -> xs; w HWIO fp32 [7][7][3][K] -> wt8; dw8 -> gw HWIO
void s2d_stem_input(const float* x, int N, int H, int W, int OH, int OW, void* xs,
                    hipStream_t st);
void s2d_stem_weight(const float* w, int K, void* wt8, hipStream_t st);
void s2d_stem_wgrad(const float* dw8, int K, float* gw, hipStream_t st);
void conv_fwd_bf16(const ConvShape& s, const float* x, const float* w, const float* bias, float* y,
                   bool relu, float* ws, hipStream_t st, const void* xb = nullptr,
                   const void* wtb = nullptr, void* yb = nullptr,
                   const ConvStats* stats = nullptr);
void conv_bwd_data_bf16(const ConvShape& s, const float* dy, const float* w, float* dx, float* ws,
                        hipStream_t st, const void* dyb = nullptr, const float* addend = nullptr,
                        const void* wtb = nullptr, const BnBwdStats* bstats = nullptr);
// batched weight re-layout: jobs = device int64 [njobs][8] = {w, out, taps,
// C, K, mode (0 bf16 forward, 1 bf16 stride-1 dgrad, 2 fp32 stride-1 dgrad:
// flipped + ci / co transposed), first block, 0}, blocks of a job
// = wcvt_blocks(taps, C, K), first blocks ascending
long long wcvt_blocks(int taps, int C, int K);
void wcvt_batch(const long long* jobs, int njobs, long long nblocks, hipStream_t st);
// flat momentum SGD (optim::sgd_momentum_flat arithmetic, l2 on every
// element) that also writes the bf16 layouts of the updated conv weights:
// jobs = device int64 [njobs][8] = {w offset (floats), forward out, dgrad out,
// taps, C, K, first block, kind} (wcvt_blocks(taps, C, K) blocks each; kind 0:
// both bf16 layouts per block, kind 1: the fp32 flipped dgrad layout); ranges = device int64 [nranges][4] = {lo4, hi4, first
// block, blocks} of the other float4 ranges (first blocks ascending, counted
// from conv_blocks); step (optional) is bumped once
void sgd_wcvt(float* w, const float* g, float* mom, float momentum, float gscale, float l2,
              const float* lr, long long* step, const long long* jobs, int njobs,
              long long conv_blocks, const long long* ranges, int nranges, long long range_blocks,
              hipStream_t st);
bool conv_bwd_filter_bf16_ok(const ConvShape& s);
void conv_bwd_filter_bf16(const ConvShape& s, const float* x, const float* dy, float* ws,
                          float* dw, hipStream_t st, const void* xb = nullptr,
                          const void* dyb = nullptr);
// LDS-tiled conv family (conv_tiled.hip), used by the launchers above for the
// shapes it supports
bool conv_fwd_tiled_ok(const ConvShape& s);
bool conv_fwd_tiled_gather_ok(const ConvShape& s);  // fp32 tiled forward, flattened (kh, kw, ci)
bool conv_bwd_data_tiled_ok(const ConvShape& s);
bool conv_bwd_filter_tiled_ok(const ConvShape& s);
void conv_fwd_tiled(const ConvShape& s, const float* x, const float* w, const float* bias, float* y,
                    bool relu, float* ws, hipStream_t st, bool bf16,
                    const ConvStats* stats = nullptr);
// partial rows of the BatchNorm statistics the tiled forward writes (fp32 route)
int conv_fwd_tiled_stats_rows(const ConvShape& s, bool bf16);
// dy may be null when dyb (bf16 dY) is given
// wflip (optional, fp32 stride-1 dgrad): the weights already flipped and
// ci / co-transposed, W'[kh][kw][co][ci] = W[R-1-kh][S-1-kw][ci][co]
// (wcvt_batch mode 2 / sgd_wcvt fp32 jobs); else a wflip launch derives them
void conv_bwd_data_tiled(const ConvShape& s, const float* dy, const float* w, float* dx, float* ws,
                         hipStream_t st, bool bf16, const float* addend = nullptr,
                         const void* dyb = nullptr, const float* wflip = nullptr);
long long conv_fwd_tiled_ws_floats(const ConvShape& s, bool epilogue);
// Tile / split plan of the tiled family.  Production runs the defaults (the
// measured choices, docs/PERF_NOTES.md); labs (scripts/conv_lab.py) change
// them through the binding before building workspaces, never per call.
struct TiledPlan {
  long long m128_min_bf16 = 128LL * 256;  // 128-row tiles from M >= this (bf16)
  long long m128_min_f32 = 1LL << 62;     // fp32: never (64-row tiles measured faster)
  int ksplit_target = 1024;               // forward / dgrad split-K: blocks to aim for
  int wgsplit_target = 1024;              // filter gradient: blocks to aim for
  int gcap = 256;                         // filter gradient slice cap, gather path
  int vcap = 256;                         // filter gradient slice cap, vector path
  bool wg_xcd = false;                    // filter gradient slices grouped by XCD (xcd_slice_bid; slower)
  bool dgrad_fwd = true;                  // fp32 stride-1 dgrad through the forward kernel
  bool wg64 = true;                       // 64-wide ci tiles for every filter gradient
  bool wg_n64 = false;                    // ... and 64-wide co tiles (labs)
  bool wg_bk16 = true;                    // fp32 64 x 128 filter tiles on 16-pixel K tiles
  bool wg_bk16_64 = false;                // ... and the 64 x 64 ones (56x56 layer 109 -> 117 us: off)
  bool halo_f32 = true;                   // fp32 3x3 stride-1 convs on conv3f_kernel
  // ... with 128-column tiles on 16-channel chunks for K % 128 == 0: measured a
  // wash (conv_lab fwd + dgrad 2292 vs 2270 us a step), so off
  bool halo_f32_wide = false;
  int halo_f32_bm = 0;                    // conv3f block rows: 0 = by grid (conv3f_plan), 64, 128
  // conv3f channels a chunk with 64 columns: 16 (64-byte rows, 38 KiB of LDS,
  // four blocks a CU) or 32 (77 KiB, two): conv_lab fwd + dgrad 2188 vs 2212 us
  // a step, ResNet-18 fp32 5.573 / 5.562 vs 5.674 / 5.680 ms (r6_s29.steps)
  int halo_f32_ch = 16;
  bool halo_f32_small = false;            // conv3f 64 x 64 / 16 ch with a 288-row halo, 3-deep ring
  bool halo_f32_s2 = true;                // fp32 3x3 stride-2 dgrad on dgrad3s2f_kernel
  // ... its split-K target (0: ksplit_target): fewer, longer slices than the
  // other convs (three blocks a CU, a dX four times the dY grid to sum):
  // ResNet-18 fp32 5.462 / 5.465 -> 5.432 / 5.416 ms at 1024 -> 512 (r6_s33.steps)
  int ksplit_s2 = 512;
};
// fp32 3x3 / stride 1 / pad 1 halo conv (conv_tiled.hip conv3f_kernel); wt:
// [9][K][C] read at tap 8 - t - the forward passes the stride-1 dgrad copy
// (wflip layout), the dgrad the HWIO weights; ws: conv3f_ws_floats
bool conv3f_ok(const ConvShape& s);
long long conv3f_ws_floats(const ConvShape& s);
void conv3f(const ConvShape& s, const float* x, const float* wt, float* y, float* ws,
            hipStream_t st, const float* addend);
TiledPlan& tiled_plan();
long long conv_bwd_data_tiled_ws_floats(const ConvShape& s);
int conv_filter_tiled_splits(const ConvShape& s);
void conv_bwd_filter_tiled(const ConvShape& s, const float* x, const float* dy, float* part,
                           float* dw, hipStream_t st, bool bf16);
// mode 0: s1 = colsum(a), s2 = colsum(a^2); mode 1: s1 = colsum(a), s2 = colsum(a*b).
// ws (chan_reduce_ws_floats) selects the deterministic bn.hip reduction;
// null falls back to memset + atomics.
void colsum2(const float* a, const float* b, long long rows, int C, float* s1, float* s2, int mode,
             float* ws, hipStream_t st);
// bn.hip: deterministic per-channel reductions and BatchNorm (C % 4 == 0,
// 4 <= C <= 1024)
bool chan_reduce_ok(int C);
long long chan_reduce_ws_floats(long long rows, int C);
void chan_reduce(const float* a, const float* b, long long rows, int C, float* s1, float* s2,
                 int mode, float* ws, hipStream_t st);
// training: batch statistics -> mean / rstd, running stats updated in place
// (momentum, unbiased var); eval: normalise with rmean / rvar.  y = BN(x)
// (+ res) (ReLU).
// x: fp32, or bf16 when xb16 (the ResNet bf16 path's conv outputs); y may be
// null when yb is given (only the bf16 twin is written)
void bn_fwd(const void* x, long long rows, int C, const float* g, const float* b,
            const float* res, float* y, float* mean, float* rstd, float* ws, float eps,
            float momentum, bool relu, bool training, float* rmean, float* rvar, hipStream_t st,
            void* yb = nullptr,  // yb: optional bf16 copy of y
            bool xb16 = false);
// training forward from the statistics a conv epilogue already wrote
// (ConvStats part [2][C][P] of (x - shift), shift = rmean before the update):
// finalize + apply only, no statistics pass over x
void bn_fwd_partials(const float* part, int P, const float* shift, const void* x, long long rows,
                     int C, const float* g, const float* b, const float* res, float* y, float* mean,
                     float* rstd, float eps, float momentum, bool relu, float* rmean, float* rvar,
                     hipStream_t st, void* yb = nullptr, bool xb16 = false);
// dg = sum dy' xhat, db = sum dy', dx, and dres = dy' (dy' = dy [y > 0] if relu);
// dx (fp32) and dxb (bf16) are each optional, at least one is required;
// y (the ReLU mask) is the fp32 output, or its bf16 twin when yb16
void bn_bwd(const void* x, const float* dy, const void* y, const float* mean, const float* rstd,
            const float* g, long long rows, int C, bool relu, float* ws, float* dg, float* db,
            float* dx, float* dres, hipStream_t st, void* dxb = nullptr, bool xb16 = false,
            bool yb16 = false);
// backward from the statistics the producing dgrad's epilogue already wrote
// (BnBwdStats part, P rows): finalize + apply only, no statistics pass;
// x bf16, y = the bf16 twin (relu)
void bn_bwd_partials(const float* part, int P, const void* x, const float* dy, const void* y,
                     const float* mean, const float* rstd, const float* g, long long rows, int C,
                     bool relu, float* dg, float* db, float* dx, float* dres, hipStream_t st,
                     void* dxb);
// bn_fwd_partials / bn_bwd_partials run the finalize inside the apply launch
// (one launch, grid-wide barrier) unless turned off (A/B, tests); the sticky
// error word is non-zero if a barrier spin ever timed out
void bn_set_fused(bool on);
unsigned bn_fused_error();
void bn_set_fused_blocks_per_cu(int bpc);
int bn_fused_grid_cap();  // blocks of a fused launch (0: fused off)
// microseconds per grid-wide barrier (grid_sync.h) of `blocks` 256-thread blocks
float gsync_barrier_us(int blocks, int iters);
void maxpool_fwd(const PoolShape& p, const float* x, float* y, int* arg, hipStream_t st);
void maxpool_bwd(const PoolShape& p, const float* dy, const int* arg, float* dx, hipStream_t st);
// bf16-twin form: xb = bf16 input, y (fp32) / yb (bf16) outputs each optional,
// arg = window-relative tap (uint8); C % 4 == 0, k * k < 255
bool maxpool_b16_ok(const PoolShape& p);
// fp32 input, uint8 window-relative taps (maxpool_bwd_b8 takes them back)
void maxpool_fwd_u8(const PoolShape& p, const float* x, float* y, uint8_t* arg, hipStream_t st);
void maxpool_fwd_b16(const PoolShape& p, const void* xb, float* y, void* yb, uint8_t* arg,
                     hipStream_t st);
void maxpool_bwd_b8(const PoolShape& p, const float* dy, const uint8_t* arg, float* dx,
                    hipStream_t st);
void avgpool_fwd(const float* x, float* y, int N, int HW, int C, hipStream_t st);
void avgpool_bwd(const float* dy, float* dx, int N, int HW, int C, hipStream_t st);
void xent(const float* logits, const int* labels, int B, int C, float* loss_rows, float* dlogits,
          int* correct, hipStream_t st);
void relu_bwd(const float* dy, const float* y, float* dx, long long n, hipStream_t st);
void softmax_rows(const float* x, float* y, int M, int N, hipStream_t st);
// stem im2col route: HWIO weight -> bf16 [K][kp] (im2col k order), and the
// [kp][K] filter gradient back to HWIO
void stem_weight_bf16(const float* w, int R, int sc, int seg, int kp, int K, void* out,
                      hipStream_t st);
void stem_wgrad(const float* gpad, int R, int sc, int seg, int K, float* gw, hipStream_t st);
// one-workgroup softmax xent with the mean loss (B rows of C classes)
void xent_mean(const float* logits, const int* labels, int B, int C, float* loss_rows,
               float* dlogits, float* mean, int* correct, hipStream_t st);
// small FC layers: y = x W (+ b) (+ ReLU); backward dW, db, dX (dX optional)
void linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int K, int N,
                bool relu, hipStream_t st);
void linear_bwd(const float* x, const float* w, const float* y, const float* dy, float* dw,
                float* db, float* dx, int M, int K, int N, bool relu, hipStream_t st);
void lr_from_step(const long long* step, int n_local, int batch, float base, float decay,
                  float* lr, hipStream_t st);
// lr_out (optional): also writes the learning rate of that step (as lr_from_step)
void gather_batch(const float* data, const int* labels, const long long* step, int n_local,
                  int batch, long long row_elems, float* xb, int* yb, hipStream_t st,
                  float lr_base = 0.f, float lr_decay = 1.f, float* lr_out = nullptr);

}  // namespace gops
