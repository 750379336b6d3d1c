/*
 * azg.h -- C ABI of the MI355X batched self-play engine (libazg.so).
 *
 * This is the drop-in boundary for the reference hot path
 *     Coach.executeEpisode -> MCTS.getActionProb -> MCTS.search
 * (Coach.py:41-90, MCTS.py:33-145).  The reference exposes it as duck-typed
 * Python objects; a maintainer binds these entry points with ctypes (see
 * INTEGRATION.md).  Plain pointers and sizes only; every device pointer is
 * caller-owned (e.g. a torch tensor's data_ptr()) and every call is ordered on
 * the HIP stream passed in (torch.cuda.current_stream().cuda_stream).  All
 * calls return 0 on success or a negative AZG_ERR_* code; azg_last_error()
 * gives the thread-local message.  One engine per device, one host thread.
 *
 * A step of the engine = one simulation for every active game slot:
 *     azg_sim_begin  -- MCTS.py:83-132  select/descend to a leaf, write its
 *                       randomly symmetrised planes (InflexionGame.py:115-122)
 *     <evaluate>     -- NNetWrapper.predict (NNet.py:78-94), batched, or
 *                       azg_stub_eval (test evaluator)
 *     azg_sim_end    -- MCTS.py:89-112 expand + MCTS.py:136-145 backup
 * and after numMCTSSims steps
 *     azg_move_end   -- MCTS.py:48-60 root policy + Coach.py:68-90 sample,
 *                       apply, terminal test, record the move.
 */
#ifndef AZG_H
#define AZG_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AZG_ABI_VERSION 1

enum azg_game_kind { AZG_GAME_INFLEXION = 1, AZG_GAME_OTHELLO = 2 };

enum azg_flags {
    AZG_FLAG_GC = 1,          /* free nodes whose turn < root turn at move end */
    AZG_FLAG_RECORD = 2,      /* keep per-move root counts (training examples)  */
    AZG_FLAG_ARENA = 4,       /* arena play: the searcher takes the argmax of the
                                 one-hot policy (MCTSPlayer, InflexionPlayers.py:88),
                                 no sampling draw (Coach.py:81)                   */
};

enum azg_opponent { AZG_OPPONENT_RANDOM = 1, AZG_OPPONENT_GREEDY = 2 };

enum azg_err {
    AZG_OK = 0,
    AZG_ERR_ARG = -1,         /* bad argument / config                          */
    AZG_ERR_HIP = -2,         /* HIP runtime error                              */
    AZG_ERR_NODE_POOL = -3,   /* a game's node pool is full (raise node_capacity)*/
    AZG_ERR_PATH = -4,        /* search path deeper than max_depth              */
    AZG_ERR_NO_ACTION = -5,   /* no valid action (MCTS.py:131 best_act = -1)   */
    AZG_ERR_STATE = -6,       /* call out of order                               */
    AZG_ERR_ACTION = -7,      /* arena: the leader's action is not valid here   */
};

typedef struct {
    int32_t game_kind;        /* AZG_GAME_INFLEXION / AZG_GAME_OTHELLO            */
    int32_t n;                /* board side: InflexionGame 7, OthelloGame 6 or 8  */
    int32_t max_turns;        /* InflexionGame max_turns (main.py:34: 343)        */
    int32_t num_games;        /* G concurrent game slots on this device           */
    int32_t sims;             /* args.numMCTSSims                                 */
    int32_t temp_threshold;   /* args.tempThreshold                               */
    double cpuct;             /* args.cpuct                                       */
    uint32_t seed_base;       /* slot i of game index k is seeded seed_base + k   */
    int32_t pad0;
    int64_t first_game;       /* global game index of slot 0 (multi-GPU shards)   */
    int32_t node_capacity;    /* nodes per game slot, 0 = default                 */
    int32_t max_depth;        /* search path capacity, 0 = default (256)          */
    int32_t max_moves;        /* recorded moves per game, 0 = max_turns + 1       */
    int32_t flags;            /* AZG_FLAG_*                                       */
} azg_config;

typedef struct azg_engine azg_engine;

/* Engine lifetime.  `stream` is a hipStream_t (may be NULL = default stream). */
int  azg_create(const azg_config* cfg, void* stream, azg_engine** out);
void azg_destroy(azg_engine* e);
const char* azg_last_error(void);
int  azg_abi_version(void);

/* Start a new generation: every slot gets a fresh game (InflexionGame.restarted,
 * Game.py:82; Coach.py:110-111 fresh MCTS) seeded with seed_base + first_game + i. */
int  azg_reset(azg_engine* e, uint32_t seed_base, int64_t first_game, void* stream);

/* One simulation step.  leaf_planes: device f32 [G,4,n,n] written by sim_begin;
 * P: device f32 [G, p_stride] (probabilities, exp of the net's log_softmax),
 * v: device f32 [G].  Slots without a leaf to evaluate get zero planes and
 * ignore P/v. */
int  azg_sim_begin(azg_engine* e, float* leaf_planes, void* stream);
int  azg_sim_end(azg_engine* e, const float* P, int32_t p_stride, const float* v, void* stream);
/* azg_sim_end of this simulation and azg_sim_begin of the next in one launch (same
 * results: one wave per slot does the backup, then the next descent); saves a kernel
 * boundary per simulation where the search is launch-bound (few slots, one leaf each). */
int  azg_sim_end_begin(azg_engine* e, const float* P, int32_t p_stride, const float* v, float* leaf_planes,
                       void* stream);

/* Test evaluator (tests/golden/stubnet.py spec): planes -> P, v on device. */
int  azg_stub_eval(azg_engine* e, const float* leaf_planes, float* P, float* v, void* stream);

/* Root policy, sampling, move application, recording, node GC. */
int  azg_move_end(azg_engine* e, void* stream);

/* Continuous batching: call after azg_move_end.  Every slot
 * whose game has ended hands its record to row j of the caller's completed-game
 * buffers (j = atomicAdd(*count, 1), completion order; only games with index <
 * end_game, and only while j < cap): ids[j] = global game index, moves[j],
 * actions / temps [j][max_moves], counts [j][max_moves][A] (NULL to skip); the
 * slot then starts global game k = atomicAdd(*next_game, 1) (seed seed_base + k,
 * fresh tree) if k < end_game, else goes idle.  next_game and count are device
 * int64 counters the caller initialises (next_game = first_game + G after
 * azg_reset).  A game's record is the same whichever slot it ran in. */
int  azg_refill(azg_engine* e, int64_t* next_game, int64_t end_game, uint32_t seed_base, int64_t* count,
                int64_t cap, int64_t* ids, int32_t* moves, int32_t* actions, int8_t* temps, int32_t* counts,
                void* stream);

/* Number of slots whose game is still ongoing (synchronises the stream). */
int  azg_active_games(azg_engine* e, int32_t* out, void* stream);

/* Host-side state access (synchronise the stream). */
int  azg_get_state(azg_engine* e, int8_t* boards /*[G,n*n]*/, int32_t* turns, int32_t* players,
                   int32_t* outcomes, int32_t* active, void* stream);
int  azg_set_root(azg_engine* e, int32_t slot, const int8_t* board /*[n*n]*/, int32_t turn,
                  int32_t player, void* stream);
int  azg_get_rng(azg_engine* e, int32_t slot, uint32_t* mt /*[624]*/, int32_t* pos, void* stream);
int  azg_set_rng(azg_engine* e, int32_t slot, const uint32_t* mt /*[624]*/, int32_t pos, void* stream);
/* The drop-in's per-call slot I/O (MCTS.getActionProb on one game) in one upload and one
 * download: azg_slot_begin = azg_set_root + azg_set_rng (no host synchronisation; the
 * engine's pinned staging buffer is reused once the previous upload has been read);
 * azg_slot_end = azg_root_counts + azg_get_rng + the slot's active flag, and returns the
 * slot's engine error (a full node pool, ...) as its code. */
int  azg_slot_begin(azg_engine* e, int32_t slot, const int8_t* board, int32_t turn, int32_t player,
                    const uint32_t* mt /*[624]*/, int32_t pos, void* stream);
int  azg_slot_end(azg_engine* e, int32_t slot, int32_t* counts /*[A]*/, uint32_t* mt /*[624]*/, int32_t* pos,
                  int32_t* active, void* stream);
int  azg_root_counts(azg_engine* e, int32_t slot, int32_t* counts /*[A]*/, void* stream);

/* Recorded moves: actions [G,max_moves], temps [G,max_moves], counts
 * [G,max_moves,A] (NULL to skip), moves made [G]. */
int  azg_read_moves(azg_engine* e, int32_t* actions, int8_t* temps, int32_t* counts,
                    int32_t* moves, void* stream);

/* Counters: [0] expansions [1] terminal hits [2] fallback expansions
 * [3] max path depth [4] max live nodes in a slot [5] error code [6] sims run */
int  azg_stats(azg_engine* e, int64_t* out /*[8]*/, void* stream);

/* Leaf-network epilogue: x[r, c] = max(x[r, c] + bias[c], 0) in place on an NHWC
 * f32 activation of `rows` pixels x `channels` (multiple of 4, 16-B aligned).
 * Replaces the BatchNorm + ReLU after each conv of InflexionNNet.forward
 * (InflexionNNet.py:42-45) once BN is folded into the conv. */
int  azg_bias_relu_nhwc(float* x, const float* bias, int64_t rows, int32_t channels, void* stream);

/* Leaf-network 3x3 convolution, stride 1, as an f32-MFMA implicit GEMM with the
 * folded-BN bias and ReLU fused (conv2-4 + bn2-4 + relu of InflexionNNet.forward,
 * InflexionNNet.py:43-45): x NHWC [batch, h_in, h_in, c_in], wt [9*c_in, c_out]
 * (k = (dy*3+dx)*c_in + c), y NHWC [batch, h_out, h_out, c_out] with
 * h_out = h_in + 2*pad - 2; c_in % 32 == 0, c_out % 128 == 0.  May allocate a
 * split-K workspace on first use of a shape (not inside a graph capture). */
int  azg_conv3x3_bias_relu_nhwc(const float* x, const float* wt, const float* bias, float* y, int32_t batch,
                                int32_t h_in, int32_t pad, int32_t c_in, int32_t c_out, void* stream);
/* Tuning hook: the same convolution with an explicit variant: 0..3 register-
 * staged A with BNxBK 128x32, 128x16, 256x16, 256x32; 4 LDS-DMA 3-slot ring
 * (128x128x16, split-K tail; the default); 5 the ring with next-stage operand
 * reads overlapping the current stage's MFMAs. */
int  azg_conv3x3_variant(int variant, const float* x, const float* wt, const float* bias, float* y, int32_t batch,
                         int32_t h_in, int32_t pad, int32_t c_in, int32_t c_out, void* stream);

/* Leaf-network 3x3 convolutions as Winograd convolutions over mixed F(5,3) /
 * F(4,3) / F(3,3) / F(2,3) tiles (azg_winograd.hip).  They replace the convolutions
 * of InflexionNNet.forward (InflexionNNet.py:39-45, BN folded).  An h-long output axis
 * is cut into the fewest tiles of side <= 5, p = ceil(h/5), sides as equal as possible
 * (big = small + 1: 7 = 4+3, 5 = 5, 3 = 3, 8 = 4+4, 6 = 3+3); azg_winograd_layout
 * returns p, writes the sides to seq[p] and the tiles per image of the groups
 * (big,big) (big,small) (small,big) (small,small) to groups[4].  azg_winograd_tables
 * copies F(m,3)'s B^T [(m+2)^2] and A^T [m(m+2)] (row-major; m = 2..5) to bt, at.
 * V and M hold the groups one after another, group g = (ma, mb) as
 * [P_g = (ma+2)(mb+2) points][batch * tiles_g][row], tiles row-major per image.
 *   azg_winograd_in_nhwc : x NHWC [batch, h_in, h_in, c] (zero padding `pad`) ->
 *                          V (B^T d B per tile and channel, format vfmt below);
 *                          with in_bias != NULL, relu(x + in_bias[c]) is
 *                          transformed (the previous layer's bias + ReLU fused);
 *   (caller)             : M_e = V_e x U_e per point e, U = G_ma g G_mb^T
 *                          (times mscale^-1, a power of two, for split V);
 *   azg_winograd_out_nhwc: M f32 (rows of k) -> y NHWC [batch, h_out, h_out, k] =
 *                          A^T (mscale M) A + bias, ReLU if relu != 0.
 * V formats: AZG_WINO_F32 f32 rows of c; AZG_WINO_SPLIT2 fp16 rows of 2c in 32-channel
 * blocks [hi(32) | lo(32)] (channel j's hi at 64 (j / 32) + j % 32, its lo 32 further;
 * c % 32 == 0; the A operand of azg_split_gemm); AZG_WINO_SPLIT fp16 rows of 3c =
 * [hi | lo | hi], hi = fp16(v), lo = fp16(v - hi) -- the A operand of the
 * error-compensated GEMM [hi|lo|hi] x [Uh; Uh; Ul] (f32 accumulation); a value
 * fp16 cannot hold (|v| > 65504, NaN) sets *overflow (device int, required: a
 * host pointer is rejected with AZG_ERR_ARG, the kernels set it with a device atomic).
 * c % 4 == 0, k % 4 == 0, 16-B aligned pointers, h_out <= 64. */
enum { AZG_WINO_F32 = 0, AZG_WINO_SPLIT = 1, AZG_WINO_SPLIT2 = 2 };
int  azg_winograd_layout(int32_t h_out, int32_t* seq, int32_t* groups);
int  azg_winograd_tables(int32_t m, float* bt, float* at);
int  azg_winograd_in_nhwc(const float* x, const float* in_bias, void* V, int32_t batch, int32_t h_in, int32_t pad,
                          int32_t c, int32_t vfmt, int32_t* overflow, void* stream);
int  azg_winograd_out_nhwc(const float* M, const float* bias, float* y, int32_t batch, int32_t h_out, int32_t k,
                           int32_t relu, float mscale, void* stream);
/* The output transform writing, instead of the NHWC activation, one row per image of
 * the flattened NHWC activation (width w = h_out*h_out*k) in split format vfmt
 * (AZG_WINO_SPLIT [hi|lo|hi] or AZG_WINO_SPLIT2 [hi|lo] blocks): the A operand of a
 * split GEMM over it (the network's fc1, InflexionNNet.py:47).  kparts > 1 cuts each
 * row into kparts chunks of w / kparts stored as kparts matrices [kparts][batch][chunk]
 * (the parts of a split-K GEMM; chunk % 32 == 0 for AZG_WINO_SPLIT2, % 4 otherwise).
 * Same checks as above; out-of-range values set *overflow. */
int  azg_winograd_out_split(const float* M, const float* bias, void* y, int32_t batch, int32_t h_out, int32_t k,
                            int32_t relu, float mscale, int32_t vfmt, int32_t kparts, int32_t* overflow,
                            void* stream);
/* Between two Winograd layers with no padding on the second (conv2->conv3->conv4):
 * M of layer i (h x h outputs, c channels) -> relu(A^T (mscale M) A + bias) -> V of
 * layer i+1 (input h x h, format vfmt) in one pass; the activation stays on chip.
 * 3 <= h <= 9, c % 64 == 0. */
int  azg_winograd_mid_nhwc(const float* M, const float* bias, void* V, int32_t batch, int32_t h, int32_t c,
                           float mscale, int32_t vfmt, int32_t* overflow, void* stream);
/* The first two layers' front end: conv1 (planes NCHW [batch, depth, n, n] ->
 * c channels, 3x3, pad 1, weights w1 [c][depth][3][3], bias b1) + ReLU, then
 * conv2's Winograd input transform (pad 1) -> V (format vfmt) in one pass.
 * depth <= 4, 3 <= n <= 9, c % 64 == 0. */
int  azg_winograd_first_nchw(const float* planes, const float* w1, const float* b1, void* V, int32_t batch,
                             int32_t depth, int32_t n, int32_t c, int32_t vfmt, int32_t* overflow, void* stream);
/* The Winograd GEMMs of one layer as an error-compensated fp16 MFMA GEMM
 * (azg_split_gemm.hip): for every point e of nruns runs (run r: points[r]
 * points with rows[r] rows each, stored one after another),
 *   M_e [rows x k] f32 = A_e x B_e^T,  A_e [rows][2c] fp16 rows of 32-channel
 *   [hi | lo] blocks (V in AZG_WINO_SPLIT2), B_e [k][2c] fp16 rows in the same blocks
 *   (U^T, points of all runs in order), computed as hi.hi + lo.hi + hi.lo with f32
 *   accumulation.  Schedule: 256 x 256 tiles (variant 4), or 128 x 256 / 64 x 256
 *   tiles (variants 17 / 18) when those need fewer rounds of the chip (small leaf
 *   batches).
 * c % 64 == 0, k % 256 == 0, nruns <= 4, 16-B aligned pointers. */
int  azg_split_gemm(const void* a, const void* bt, float* m, int32_t nruns, const int32_t* points,
                    const int32_t* rows, int32_t c, int32_t k, void* stream);
/* The same with an explicit kernel schedule, for tests: 0 (reads, then MFMAs per stage,
 * one tile per workgroup), 4 (variant 0 persistent, the azg_split_gemm default), 17 / 18
 * (variant 0 on 128 / 64-row tiles, azg_split_gemm's pick for short launches).  The
 * probe-only schedules measured in HISTORY.md (1-3, 5-8, 10-12, 15, 16, 19) are not in the
 * product library: tools/Makefile builds them into tools/libazg_probes.so, which exports this
 * entry point for all of them and azg_split_gemm_stamps (per-wave phase stamps of variant 4);
 * other values return AZG_ERR_ARG here. */
int  azg_split_gemm_variant(int32_t variant, const void* a, const void* bt, float* m, int32_t nruns,
                            const int32_t* points, const int32_t* rows, int32_t c, int32_t k, void* stream);
/* The leaf network at one to four leaves (azg_small.hip; InferenceNet's forward below
 * SMALL_MAX_B leaves, the drop-in MCTS's batch-1 search), one launch per layer, f32 with a
 * fixed summation order:
 *   azg_small_conv3x3: y[px * ldy + co] = relu?(bias[co] + sum_k w[co][k] x_im2col[k][px]),
 *     k = tap * Cin + ci, w [Cout][3][3][Cin] (a channels_last conv weight, BN folded),
 *     px = (leaf, oy, ox) of the (H + 2 pad - 2)^2 output, x any layout given by its
 *     element strides (sB per leaf, sY, sX, sC: the NCHW leaf planes or the NHWC rows this
 *     writes); Cout even, at most 256 output pixels, pad 0 or 1; bias may be null.  With a
 *     device workspace (work: >= 8 Cout x batch x (output pixels) floats, 16-B aligned;
 *     tickets: >= Cout / 8 zero-initialised words, left zero after every launch), NHWC
 *     float4 inputs with Cin % 32 == 0, Cout % 8 == 0 and more than 16 output pixels, the
 *     split-K form runs (8 channels x an eighth of the input channels per block, the eighths
 *     summed in order by the last block of each channel group); else work / tickets may be null;
 *   azg_small_fc: y[b * ldy + n] = relu?(bias[n] + sum_k w[n][k] x[b * ldx + k]), b < batch <= 4,
 *     w [N][K] row-major, K % 4 == 0, ldx % 4 == 0, x and w 16-B aligned; bias may be null. */
int  azg_small_conv3x3(const float* x, int64_t sB, int32_t sY, int32_t sX, int32_t sC, int32_t batch, int32_t H,
                       int32_t pad, const float* w, int32_t Cin, int32_t Cout, const float* bias, int32_t relu,
                       float* y, int32_t ldy, float* work, int64_t work_floats, uint32_t* tickets,
                       int32_t n_tickets, void* stream);
int  azg_small_fc(const float* x, int32_t ldx, int32_t batch, const float* w, int32_t K, int32_t N, const float* bias,
                  int32_t relu, float* y, int32_t ldy, void* stream);
/* conv1 + conv2 at one to four leaves in one launch (the split-K form of azg_small_conv3x3, each
 * block computing relu(b1 + conv1(planes)) for its quarter of conv2's input channels itself):
 * planes [batch][depth][n][n] f32 (depth <= 4, the boards' sides 6 <= n <= 8), w1 [C][3][3][depth], w2 [C][3][3][C]
 * (channels_last, BN folded), y[px * ldy + co] = relu(b2 + conv2(...)) for the n x n outputs;
 * C % 16 == 0, work / tickets as azg_small_conv3x3's split-K form (4 K-parts here). */
int  azg_small_conv12(const float* planes, int32_t batch, int32_t depth, int32_t n, const float* w1, const float* b1,
                      const float* w2, const float* b2, int32_t C, float* y, int32_t ldy, float* work,
                      int64_t work_floats, uint32_t* tickets, int32_t n_tickets, void* stream);
/* [fc3 | fc4] and the heads in one launch (1-4 leaves): logits[b][n] = sum_k w34[n][k] x[b][k]
 * for n <= A, then P[b] = softmax(b34[:A] + logits[b][:A]), v[b] = tanh(b34[A] + logits[b][A])
 * (azg_policy_value's arithmetic) by the last block to finish; *ticket zero before and after. */
int  azg_small_heads(const float* x, int32_t ldx, int32_t batch, const float* w34, int32_t K, int32_t A,
                     const float* b34, float* logits, float* P, float* v, uint32_t* ticket, void* stream);
/* The schedule azg_split_gemm picks for a launch of this shape (4, 17 or 18). */
int  azg_split_gemm_pick(int32_t nruns, const int32_t* points, const int32_t* rows, int32_t k);
/* Cap the persistent split GEMM's grid at `blocks` workgroups (one per CU; 0 = every CU;
 * rounded down to a multiple of 8, at least 8: one per XCD tile range), process-wide, so
 * that a second stream's kernels (the other half-batch's transforms) find CUs free
 * beside it.  Results do not depend on it. */
int  azg_set_gemm_blocks(int32_t blocks);

/* The fully connected tail of the leaf network (InflexionNNet.py:47-54, BN folded)
 * around split-fp16 GEMMs (azg_heads.hip; the GEMMs are the caller's -- libazg's azg_split_gemm
 * in the default forms (split-K parts in AZG_WINO_SPLIT2 layout, azg_fc_act / azg_fc_act_t /
 * azg_policy_value_parts below), or one fp16 GEMM per layer with f32 accumulation over A rows
 * [hi | lo | hi] times the weights stacked [hi; hi; lo] (the AZG_WINO_SPLIT forms, split_blas),
 * pre-scaled by a power of two that `scale` undoes).
 *   azg_fc_act_split: y = bias + scale * sum_p m[p] (parts >= 1 partial products
 *                     [rows][n] f32, part p at m + p * part_stride floats: the parts of a
 *                     split-K GEMM, summed in order), ReLU if relu != 0, written as the
 *                     next GEMM's A operand: fp16 rows [hi(n) | lo(n) | hi(n)]
 *                     (AZG_WINO_SPLIT); |y| > 65504 or NaN sets *overflow.
 *                     n % 4 == 0, part_stride % 4 == 0; m, bias 16-B and out 8-B aligned.
 *   azg_policy_value: P[r][a] = softmax_a(bias[a] + scale * m[r][a]) (a < actions,
 *                     = exp(log_softmax), NNet.py:94) and v[r] = tanh(bias[actions] +
 *                     scale * m[r][actions]) from the stacked [fc3 | fc4] output m
 *                     (row stride ldm >= actions + 1); P [rows][actions], v [rows].
 *                     actions <= 1024. */
int  azg_fc_act_split(const float* m, int32_t parts, int64_t part_stride, const float* bias, float scale, void* out,
                      int32_t rows, int32_t n, int32_t relu, int32_t* overflow, void* stream);
int  azg_policy_value(const float* m, int32_t ldm, const float* bias, float scale, float* P, float* v,
                      int32_t rows, int32_t actions, void* stream);
/* The same epilogues for an FC tail that runs entirely on azg_split_gemm (no library
 * GEMM): azg_fc_act writes y as fmt AZG_WINO_SPLIT ([hi | lo | hi] rows, out_parts 1,
 * = azg_fc_act_split) or AZG_WINO_SPLIT2: out_parts K-parts of 32-channel [hi | lo]
 * blocks, [part][rows][2 n / out_parts] fp16 -- the A operand of the next layer's
 * split-K azg_split_gemm (its parts as the GEMM's points); (n / out_parts) % 32 == 0.
 * azg_policy_value_parts sums `parts` (1..16) partial [fc3 | fc4] products (part p at m + p *
 * part_stride floats, in order) first; azg_policy_value = parts 1. */
int  azg_fc_act(const float* m, int32_t parts, int64_t part_stride, const float* bias, float scale, void* out,
                int32_t rows, int32_t n, int32_t relu, int32_t fmt, int32_t out_parts, int32_t* overflow,
                void* stream);
int  azg_policy_value_parts(const float* m, int32_t parts, int64_t part_stride, int32_t ldm, const float* bias,
                            float scale, float* P, float* v, int32_t rows, int32_t actions, void* stream);
/* azg_fc_act (AZG_WINO_SPLIT2 output) for TRANSPOSED partial products m [parts][n][rows] (the
 * small-batch fc1 computed as W x A^T, every weight tile read once); rows % 64 == 0, n % 64 == 0,
 * (n / out_parts) % 64 == 0, 1 <= parts <= 32.  Same arithmetic: y = bias + scale * (parts summed in order). */
int  azg_fc_act_t(const float* m, int32_t parts, int64_t part_stride, const float* bias, float scale, void* out,
                  int32_t rows, int32_t n, int32_t relu, int32_t out_parts, int32_t* overflow, void* stream);

/* Device pointers of the engine state (for zero-copy consumers, e.g. the
 * example gather): [0] boards i8 [1] turns [2] players [3] outcomes [4] active
 * [5] record actions [6] record counts [7] moves */
int  azg_device_ptrs(azg_engine* e, void** out /*[8]*/);

/* Batched Arena (Arena.py:38-142 with MCTSPlayer vs a baseline player,
 * Coach.py:158-165).  After azg_reset, azg_set_arena gives every slot the
 * colour the search plays (searcher[g] = +1 RED / -1 BLUE) and the colour to
 * move first (first_player[g], Arena.playGame's game.player = player1).  The
 * engine then searches (sim_begin / sim_end / move_end, with temp_threshold 0)
 * only in slots where the searcher is to move, and azg_opponent_move plays the
 * baseline's move (AZG_OPPONENT_RANDOM: RandomPlayer, np.random.choice of the
 * valid actions on the slot's stream; AZG_OPPONENT_GREEDY: GreedyPlayer,
 * InflexionPlayers.py:61-74) in the others.  Needs AZG_FLAG_ARENA. */
int  azg_set_arena(azg_engine* e, const int32_t* searcher /*[G] host*/, const int32_t* first_player /*[G] host*/,
                   void* stream);
int  azg_opponent_move(azg_engine* e, int32_t kind, void* stream);
/* Arena between two searchers (Arena.py:23-88 with two MCTSPlayers; replaces the
 * reference's per-game Arena.playGame loop for player1 = MCTSPlayer(net 1),
 * player2 = MCTSPlayer(net 2)).  Two arena engines hold the same games, one searching
 * for RED, the other for BLUE; after the leader's move (sim_begin / sim_end /
 * move_end), azg_arena_follow plays the leader's action in e's copy of every slot
 * where the leader just moved and gives e the leader's numpy stream for the slot (the
 * reference's two players draw from one process-wide stream).  An action that is not
 * valid in e's copy sets the slot's error (Arena.py:64-67). */
int  azg_arena_follow(azg_engine* e, const azg_engine* leader, void* stream);

/* Sizes of a supported game: out[0] cells, [1] actions (max_actions), [2] NN
 * input planes, [3] forms returned by game.symmetries(). */
int  azg_game_info(int32_t game_kind, int32_t n, int32_t* out /*[4]*/);

/* Training examples from compact move records -- Coach.executeEpisode's
 * example list (Coach.py:74-90) with game.symmetries() (InflexionGame.py:102-113)
 * for every finished game, in the reference's order (game, move, symmetry form),
 * keeping the LAST maxlen like the per-iteration deque(maxlen=maxlenOfQueue)
 * (Coach.py:107).  Records (device): moves [G], actions [G,max_moves], root visit
 * counts [G,max_moves,A] as int16 (counts_bytes 2) or int32 (4) -- what
 * azg_read_moves / the rank gather hold.  Each game is replayed from the initial
 * position; a record that is not a legal game fails with AZG_ERR_ARG; unfinished
 * games (moves < max_moves cap) contribute nothing.  Outputs (device, f32, as the
 * trainer reads them, NNet.py:54-56): planes [maxlen, planes, n, n], pis
 * [maxlen, A] (counts / sum in f64 for temp 1, one-hot of the played action for
 * temp 0), vs [maxlen] (+-outcome value).  label_mode 0 labels as Coach.py:79
 * does (player list grown by the cumulative example count), 1 labels each
 * example with its own move's player.  *count = examples written.  Synchronises
 * the stream. */
int  azg_examples(int32_t game_kind, int32_t n, int32_t max_turns, int32_t temp_threshold, int32_t num_games,
                  int32_t max_moves, const int32_t* moves, const int32_t* actions, const void* counts,
                  int32_t counts_bytes, int32_t label_mode, int64_t maxlen, float* planes, float* pis,
                  float* vs, int64_t* count, void* stream);
/* The same with counts of count_rows moves per game ([G, count_rows, A]; count_rows >= temp_threshold - 1,
 * the moves played at temperature 1 -- the only ones whose counts an example reads): the rank gather's
 * truncated records (dist.py) without a dense [G, max_moves, A] buffer.  azg_examples = count_rows
 * max_moves. */
int  azg_examples_rows(int32_t game_kind, int32_t n, int32_t max_turns, int32_t temp_threshold, int32_t num_games,
                       int32_t max_moves, const int32_t* moves, const int32_t* actions, const void* counts,
                       int32_t count_rows, int32_t counts_bytes, int32_t label_mode, int64_t maxlen, float* planes,
                       float* pis, float* vs, int64_t* count, void* stream);

/* ---- trainer convolutions (azg_wino_train.hip; NNetWrapper.train, NNet.py:36-76) ------------
 * conv2-4 of the training forward and backward on the Winograd transforms and the split GEMM
 * (azg_amd/wino_train.py drives them; replaces the MIOpen convolutions torch runs for
 * InflexionNNet.py:39-45 and their autograd).  Device pointers, caller's stream, no sync.
 *   azg_absmax          : *out = bits of max |x| over n floats (n % 4 == 0; *out zeroed first).
 *   azg_wt_u_build      : U_e = G_a w G_b^T of conv weights w [k][c][3][3] for an h_out-side
 *                         output (nnet._winograd_u's point order), scaled by 2^ku (max |U| 2^ku
 *                         in (512, 1024], *uamax = bits of max |U|), split into AZG_WINO_SPLIT2
 *                         rows: ut [P][k][2c] (the forward GEMM's B operand) and/or un
 *                         [P][c][2k] (the input-gradient GEMM's); c % 64 == k % 64 == 0; work:
 *                         ceil(c k / 256) floats (pass 1's block maxima of |U|; pass 2 recomputes U
 *                         per 32 x 32 tile from the weights -- no f32 copy of U).
 *   azg_wt_out          : y NHWC = bias + 2^-ku A^T M A (no ReLU), h_out in {3, 5, 7}.
 *   azg_wt_dout         : dM [P][T][2k] AZG_WINO_SPLIT2 = 2^kd A dy A^T (dy NHWC; 2^kd puts
 *                         max |dy| in (16, 32]); |dM| > 65504 sets *overflow.
 *   azg_wt_din          : dx NHWC [batch, h_in, h_in, c] = 2^-(kd+ku) sum over tiles of
 *                         B dV B^T (dV f32 [P][T][c]); (h_in, pad) in {(7,1), (7,0), (5,0)}.
 *   azg_wt_split2_transpose: AZG_WINO_SPLIT2 [points][t][2c] -> [points][c][2t] (t, c % 64).
 *   azg_wt_pow2_scale   : *out = the power of two the kernels scale by for amax, target. */
int  azg_absmax(const float* x, int64_t n, uint32_t* out, void* stream);
/* The trainer's BatchNorm2d + ReLU on channels-last activations x [rows][C] (rows = batch x H x W;
 * C % 4 == 0, C <= 1024), training mode (azg_train_bn.hip): azg_bn_relu_fwd writes y = relu(bn(x))
 * with the batch's statistics, sv [4C] = (scale, beta, mean, invstd), and updates run_mean /
 * run_var (momentum; unbiased variance; either may be null); azg_bn_relu_bwd writes dx, dgamma,
 * dbeta from dy (the gradient of y), x and sv.  Sums in f64 over 512 fixed row ranges, reduced in
 * order (deterministic); work >= 1026 C doubles, co >= 2C floats (scratch). */
int  azg_bn_relu_fwd(const float* x, int64_t rows, int32_t C, const float* gamma, const float* beta, float eps,
                     float momentum, float* run_mean, float* run_var, float* y, float* sv, double* work,
                     void* stream);
int  azg_bn_relu_bwd(const float* x, const float* dy, int64_t rows, int32_t C, const float* sv, float* dx,
                     float* dgamma, float* dbeta, float* co, double* work, void* stream);
/* The same in two halves around a caller's reduction over data-parallel ranks: azg_bn_sums writes
 * sums [2C] f64 = (sum x, sum x^2) of this rank's rows, azg_bn_relu_fwd_from_sums finishes from the
 * (all-reduced) sums over n_total rows; azg_bn_relu_bwd_sums writes (sum g, sum g xhat), and
 * azg_bn_relu_bwd_from_sums writes dx from the all-reduced ones (dgamma / dbeta may be null: a rank's
 * own share comes from its un-reduced sums).  work >= 1024 C doubles (azg_bn_relu_fwd / _bwd: 1026 C). */
int  azg_bn_sums(const float* x, int64_t rows, int32_t C, double* sums, double* work, void* stream);
int  azg_bn_relu_fwd_from_sums(const float* x, int64_t rows, int32_t C, const double* sums, int64_t n_total,
                               const float* gamma, const float* beta, float eps, float momentum, float* run_mean,
                               float* run_var, float* y, float* sv, void* stream);
int  azg_bn_relu_bwd_sums(const float* x, const float* dy, int64_t rows, int32_t C, const float* sv, double* sums,
                          double* work, void* stream);
int  azg_bn_relu_bwd_from_sums(const float* x, const float* dy, int64_t rows, int32_t C, const float* sv,
                               const double* sums, int64_t n_total, float* dx, float* dgamma, float* dbeta,
                               float* co, void* stream);
/* The convolution backward's statistics of its output gradient dy [rows][C] f32 (C % 4 == 0, C <= 1024,
 * rows >= 2, 16-B aligned) in one read: *amax = bits of max |dy| (what azg_wt_dout / azg_wt_din scale by)
 * and, when db is not null, db [C] = dy summed over the rows (the conv bias's gradient; f64 partials
 * over 512 fixed row ranges, summed in order).  work >= 2 * 512 * C doubles + 512 floats. */
int  azg_wt_dy_stats(const float* dy, int64_t rows, int32_t C, uint32_t* amax, float* db, double* work, void* stream);
/* The trainer's conv1 (InflexionNNet.py:39: 3x3, stride 1, padding 1, on the board planes;
 * azg_train_conv1.hip): x NHWC [batch][n][n][depth] (the planes channels_last), w [K][depth][3][3],
 * depth <= 8, n <= 8, K % 64 == 0, batch <= 262140.  azg_conv1_train_fwd writes y NHWC [batch][n][n][K] = conv + bias
 * (bias may be null); azg_conv1_train_wgrad writes dw [K][depth][3][3] and db [K] (may be null) from
 * dy NHWC [batch][n][n][K], f64 partials in a fixed order (deterministic); work >= 64 K (9 depth + 1)
 * doubles.  (No input gradient: the planes need none.) */
int  azg_conv1_train_fwd(const float* x, int64_t batch, int32_t depth, int32_t n, const float* w, const float* bias,
                         int32_t K, float* y, void* stream);
int  azg_conv1_train_wgrad(const float* x, const float* dy, int64_t batch, int32_t depth, int32_t n, int32_t K,
                           float* dw, float* db, double* work, void* stream);
int  azg_wt_u_build(const float* w, int32_t c, int32_t k, int32_t h_out, uint32_t* uamax, void* ut, void* un,
                    float* work, void* stream);
int  azg_wt_out(const float* M, const float* bias, float* y, int32_t batch, int32_t h_out, int32_t k,
                const uint32_t* uamax, void* stream);
int  azg_wt_dout(const float* dy, void* dM, int32_t batch, int32_t h_out, int32_t k, const uint32_t* dyamax,
                 int32_t* overflow, void* stream);
int  azg_wt_din(const float* dV, float* dx, int32_t batch, int32_t h_in, int32_t pad, int32_t c,
                const uint32_t* uamax, const uint32_t* dyamax, void* stream);
int  azg_wt_split2_transpose(const void* src, void* dst, int32_t points, int32_t t, int32_t c, void* stream);
int  azg_wt_pow2_scale(const uint32_t* amax, float target, float* out, void* stream);
/* dw [k][c][3][3] = 2^-kd sum_e G_a^T dU_e G_b from dU [P][c][k] (the weights' adjoint transform). */
int  azg_wt_dw(const float* dU, int32_t c, int32_t k, int32_t h_out, const uint32_t* dyamax, float* dw, void* stream);

/* ---- the training step's heads and losses (azg_train_loss.hip; NNet.py:57-61, 96-100) ---------------
 * azg_train_loss_fwd: out[0] = l_pi = -sum_b sum_a t_pi[b][a] log_softmax(x3[b])[a] / B, out[1] = l_v =
 *   sum_b (t_v[b] - tanh(z4[b]))^2 / B (rows summed in a fixed order); rows [B][4] receives each row's two
 *   terms and its softmax statistics (max, log sum exp) for the backward.
 * azg_train_loss_bwd: dx3 = g[0] (softmax(x3) sum_a t_pi - t_pi) / B and dz4 = g[1] (-2 (t_v - v)) (1 - v^2) / B
 *   (the adjoints of log_softmax and tanh as torch forms them), g: the losses' gradients (device, 2 floats).
 * x3 / t_pi / dx3 rows of A floats at strides ld3 / ldt / lddx; z4 / dz4 at strides ld4 / lddz. */
int  azg_train_loss_fwd(const float* x3, int32_t ld3, const float* z4, int32_t ld4, const float* tpi, int32_t ldt,
                        const float* tv, int32_t B, int32_t A, float* rows, float* out, void* stream);
int  azg_train_loss_bwd(const float* x3, int32_t ld3, const float* z4, int32_t ld4, const float* tpi, int32_t ldt,
                        const float* tv, const float* rows, int32_t B, int32_t A, const float* g, float* dx3,
                        int32_t lddx, float* dz4, int32_t lddz, void* stream);

/* ---- the trainer's optimizer (azg_adam.hip) -------------------------------------------------
 * azg_adam_step: torch.optim.Adam's step (NNet.py:37; the capturable foreach arithmetic of
 * torch/optim/adam.py in f32, no weight decay / amsgrad) over nseg parameter tensors in one launch:
 * params[i] / grads[i] device f32 pointers of counts[i] elements (host arrays of pointers); m, v
 * flat f32 state buffers, 16-B aligned, segment i at offset sum_{j<i} round_up(counts[j], 4);
 * *step a device f32 step counter, incremented by this call before the update (t = *step + 1).
 * 1 <= nseg <= AZG_ADAM_MAX_SEG.  The segment table is a by-value kernel argument: a launch
 * captured in a HIP graph replays with the pointers it was captured with. */
#define AZG_ADAM_MAX_SEG 48
int  azg_adam_step(int32_t nseg, float* const* params, const float* const* grads, const int64_t* counts,
                   float* m, float* v, float* step, double lr, double beta1, double beta2, double eps,
                   void* stream);

/* ---- learn-loop host helpers (azg_host.cpp; no device work) ---------------------------------
 * azg_py_shuffle: Python's random.shuffle (Lib/random.py: for i from n-1 down to 1, j =
 * _randbelow(i + 1) by getrandbits rejection, swap) of x[0..n) in place, on the MT19937 state of
 * the interpreter's `random` module: mt = random.getstate()[1][:624], *pos = its index, both
 * advanced as the interpreter would; n < 2^32.  Replaces Coach.py:149's shuffle(trainExamples)
 * over the example history (the permutation of list(range(n)) random.shuffle gives). */
int  azg_py_shuffle(int64_t* x, int64_t n, uint32_t* mt, int32_t* pos);

#ifdef __cplusplus
}
#endif
#endif
