// Host launchers of the bf16 MNIST kernel set (mnist_bf16.hip, BASELINE config
// 2: "2-layer MNIST CNN bf16 on 1xMI355X").
//
// Numerics: fp32 master weights / momentum / gradients (flat buffers, as in
// the fp32 engine); activations and activation gradients stored in bf16;
// every GEMM on v_mfma_f32_32x32x16_bf16 with fp32 accumulation; bf16 weight
// shadows re-derived from the fp32 master weights at the start of each step.
//
// bf16 tensor layouts: every MFMA operand is stored "K-packed", [K/16][rows]
// [16], so one K-step's fragments of a 32-row tile (lane l reads 8 elements
// at row l&31, k-offset 8(l>>5)) form one contiguous 1 KB read per wave.
// Padded images are zero-bordered and only their interiors are ever written,
// so the fragment fetches need no bounds checks.  B = batch rows (eval: the
// chunk rounded up to 8).
//   a1p  [2][B][18][18][16]   pooled conv1 out, ci = 16 s + c, 2-pixel border
//   a1t  [B][18][32][24]      the same as [n][Y][ci][X] (filter-grad A operand)
//   a2p  [196][B][16]         pooled conv2 out, i = (py*7+px)*64+co = 16 k + c
//   a2t  [B/16][3136][16]     transposed a2 (dW1 A operand)
//   dh16 [32][B][16]          grad at the fc1 output, j = 16 k + c
//   dht  [B/16][512][16]      transposed dh (dW1 B operand)
//   dy2p [4][B][18][18][16]   grad at the conv2 output (pre-pool), co = 16 k + c
//   dy2t [B][14][64][16]      the same as [n][y][co][x], columns 14/15 zero
//   w2t  [25][2][64][16]      conv2 W as B[k=ci][n=co] per tap
//   w2b  [25][4][32][16]      conv2 W as B[k=co][n=ci] per tap
//   w1t  [196][512][16]       fc1 W as B[k=i][n=j]
//   w1b  [32][3136][16]       fc1 W as B[k=j][n=i]
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "mnist.h"

namespace mnist16 {
// fp32 master weights -> the four bf16 shadows
void launch_shadows(const float* w1, const float* w2, uint16_t* w1b, uint16_t* w1t,
                    uint16_t* w2t, uint16_t* w2b, hipStream_t s);
// conv2 + bias + ReLU + 2x2 maxpool (+argmax); batch % 8 == 0.  a2t / idx2
// optional (eval passes null).
void launch_conv2_fwd(const uint16_t* a1p, int batch, const uint16_t* w2t, const float* b2,
                      uint16_t* a2p, uint16_t* a2t, uint8_t* idx2, hipStream_t s);
// fc1 train: split-K partial slabs part[z][B][512] (z < mnist::FC1_SPLITS)
void launch_fc1_fwd_train(const uint16_t* a2, const uint16_t* w1t, int batch, float* part,
                          hipStream_t s);
// fc1 eval: h = dropout(relu(a2 W1 + b)) fp32 [M][512]; a2p holds ld >= M rows
void launch_fc1_fwd_eval(const uint16_t* a2p, int ld, const uint16_t* w1t, const float* b, int M,
                         float* h, uint32_t key, float keep_prob, hipStream_t s);
// fc1 backward: dX (+pool2/ReLU2 scatter into dy2p / dy2t) | dW1 | fc2 grads
void launch_fc1_bwd(const uint16_t* a2, const uint16_t* a2t, const uint8_t* idx2,
                    const uint16_t* dh16, const uint16_t* dht16, const float* hd, const float* dh,
                    const float* dlog, const uint16_t* w1b, int batch, float* g_w3, float* g_b3,
                    float* g_w4, float* g_b4, uint16_t* dy2p, uint16_t* dy2t, hipStream_t s);
// conv2 bwd-data with the ReLU1 mask: da1m fp32 [B][14][14][32]
void launch_conv2_bwd_data(const uint16_t* dy2p, const uint16_t* w2b, const uint16_t* a1p,
                           int batch, float* da1m, hipStream_t s,
                           const mnist::FcSgdArgs* fc_sgd = nullptr);
// conv2 bwd-filter partial slabs part2[G][800][64] + db2 partials [4G][64]
int conv2_filter_groups(int batch);
void launch_conv2_bwd_filter(const uint16_t* a1t, const uint16_t* dy2t, int batch, float* part2,
                             hipStream_t s,
                             const mnist::C1FilterArgs* c1 = nullptr);
size_t part2_floats(int batch);
// the whole conv2 backward in one launch: filter-grad slabs (as above), da1m
// (as launch_conv2_bwd_data), the conv1 filter-grad partials of c1 (one part1
// row per 128 pooled pixels: conv2_bwd_conv1_rows) and the optional
// single-rank FC SGD
int conv2_bwd_conv1_rows(int batch);
// labs: per-block [start, end] 100 MHz clock stamps of launch_conv2_bwd into p
// (2 x blocks u64; null turns them off)
void set_conv2_bwd_prof(unsigned long long* p);
void launch_conv2_bwd(const uint16_t* dy2p, const uint16_t* w2b, const uint16_t* a1p,
                      const uint16_t* a1t, const uint16_t* dy2t, int batch, float* da1m,
                      float* part2, hipStream_t s, const mnist::FcSgdArgs* fc_sgd,
                      const mnist::C1FilterArgs* c1);
}  // namespace mnist16
