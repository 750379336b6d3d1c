/* azg_small_probes.h -- the small-batch forms that measured slower than the product's per-layer
 * VALU kernels (azg_small.hip), kept as a probe library for the record and the bit-identity tests:
 * tools/libazg_small_probes.so (tools/Makefile; azg_small.hip with -DAZG_SMALL_PROBES +
 * azg_small_mfma.hip), loaded by tools/small_probes.py.  The product library does not export them.
 *
 *   azg_small_net: one-launch forward, 125-130 us vs 65-69 us per one-leaf forward (round 5)
 *   azg_small_conv_mfma: f32-MFMA 3x3 layers, conv12 26.5 vs 19.2 us, conv3 16.9 vs 18.0, conv4 17.2
 *   vs 9.3 (round 6, profiles/r06_small_layer_bench.json)
 */
#ifndef AZG_SMALL_PROBES_H
#define AZG_SMALL_PROBES_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* The whole small-batch forward (conv1 + conv2, conv3, conv4, fc1, fc2, [fc3 | fc4] + softmax / tanh)
 * in ONE launch: the blocks of the per-layer entry points above (same arithmetic and summation
 * orders: bit-identical P, v) as the items of one in-order work queue over a grid of one 512-thread
 * block per CU, an item of layer L waiting for layer L-1's done count -- correct whatever number of
 * the blocks is resident at once (no grid barrier).  sched: 8 u32 counters, zero before the first
 * launch, left zero by every launch; a wait of ~2^24 polls gives up and sets *err (zero sched then).  w: 14 device pointers w1 b1 w2 b2 w3 b3 w4 b4
 * fw1 fb1 fw2 fb2 fw34 fb34 (BN folded; the layouts azg_small_conv12 / conv3x3 / fc / heads take);
 * acts >= batch (n^2 C + (n-2)^2 C + (n-4)^2 C + n1 + n2 + actions + 1) floats; batch <= 4, 6 <= n <= 8,
 * pads 1, 1, 0, 0 (the boards' nets); work / tickets as azg_small_conv12's (n_tickets >= C / 8 + 1). */
int  azg_small_net(const float* planes, int32_t batch, int32_t depth, int32_t n, int32_t C, int32_t actions,
                   int32_t n1, int32_t n2, const float* const* w, float* acts, int64_t acts_floats, float* P, float* v,
                   float* work, int64_t work_floats, uint32_t* tickets, int32_t n_tickets, uint32_t* sched, int32_t* err,
                   void* stream);
/* azg_small_net's grid, process-wide: `blocks` workgroups (0 = one per CU, the default; larger
 * values are capped at the CU count).  Results do not depend on it (the tests run 1 to 256). */
int  azg_small_net_blocks(int32_t blocks);
/* The 3x3 layers of the small-batch forward on the f32 MFMA (azg_small_mfma.hip): the same arithmetic
 * as azg_small_conv12 / azg_small_conv3x3 -- the same K-parts, slices and in-order sums of the same
 * fmaf chains (v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain per output) -- so bit-identical
 * outputs, spread over 16-channel x 16-row tiles.  azg_small_mfma_layout writes out[4] = (KG parts,
 * KSL slices per part, float4 steps per slice, padded steps TP) for the layer (conv12 != 0: conv2 with
 * conv1 fused); azg_small_conv_mfma takes the weights packed [KG][Cout][KSL][4][TP] (part q, channel
 * co, slice s, slot j, step t: k = 4 (s per + t) + j of the part's tap-major K = tap * (Cin / KG) + ci;
 * nnet.pack_small_mfma), x as azg_small_conv3x3's NHWC rows (sB, sY, sX; channels contiguous) or, with
 * w1 / b1 / D given, the NCHW leaf planes with conv1 (w1 [Cin][3][3][D], channels_last, BN folded)
 * computed in the kernel; y[row * ldy + co] = relu?(bias + the sums), rows = leaf x output pixel.
 * work >= tiles x max(KG, KSL) x 256 floats, tickets >= tiles zero words (left zero), tiles = ceil(batch x
 * Ho^2 / 16) x Cout / 16; batch <= 4, Cout % 16 == 0; slice lengths of 36 or 9 float4 steps (the boards'
 * layers; others AZG_ERR_ARG). */
int  azg_small_mfma_layout(int32_t H, int32_t pad, int32_t Cin, int32_t Cout, int32_t conv12, int32_t* out /*[4]*/);
int  azg_small_conv_mfma(const float* x, int64_t sB, int32_t sY, int32_t sX, int32_t batch, int32_t H, int32_t pad,
                         const float* wm, int32_t Cin, int32_t Cout, const float* bias, int32_t relu, float* y,
                         int32_t ldy, float* work, int64_t work_floats, uint32_t* tickets, int32_t n_tickets,
                         const float* w1, const float* b1, int32_t D, void* stream);

#ifdef __cplusplus
}
#endif
#endif
