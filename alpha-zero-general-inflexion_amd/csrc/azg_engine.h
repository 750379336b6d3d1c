// azg_engine.h -- device-side state of the batched self-play engine.
//
// Everything lives in HBM as structure-of-arrays indexed by game slot g (and
// node id within the slot's pool).  One 64-lane wavefront owns one game slot
// in every kernel, so no two waves ever touch the same slot's tree: the
// reference's sequential per-game semantics (MCTS.py) are preserved exactly and
// no atomics are needed on the tree.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace azg {

constexpr int WAVE = 64;
constexpr int MT_N = 624;
constexpr int MAX_POWER_AT_SPAWN = 48;   // InflexionGame.py:69

enum Outcome : int { ONGOING = 0, DRAW = 1, WON = 2, LOST = 3 };
enum LeafKind : int { LEAF_NONE = 0, LEAF_EXPAND = 1, LEAF_TERMINAL = 2 };

// A node's key (own-pieces mask, opponent mask, turn, can_spawn) and visit count
// Ns in one 32-B record: a lookup's key compare, an expansion's key writes and a
// backup step's Ns update each touch one 32-B sector instead of one per field.
struct alignas(32) NodeKey {
    uint64_t own, opp;
    int32_t turn, cs, Ns, pad;
};

// Game-specific sizes (cells, actions A, row stride = A rounded up to 64,
// planes) are compile-time constants of the game traits in azg_kernels.hip;
// the host sees them through GameOps (azg_launch.h).
struct Dev {
    int G, M, H, DMAX, max_moves;
    int max_turns, sims, temp_threshold, flags;
    float cpuct_f;

    // per slot
    int8_t* board;       // [G][64]
    int32_t* turn;       // [G]
    int32_t* player;     // [G]  +1 RED, -1 BLUE
    int32_t* outcome;    // [G]  Outcome w.r.t. player to move
    int32_t* active;     // [G]
    int32_t* searcher;   // [G]  colour the search plays (arena), 0 = both (self-play)
    int32_t* root_id;    // [G]  node id of the root during a move, -1 = look it up
    uint32_t* mt;        // [G][624]  numpy legacy MT19937 state
    int32_t* mt_pos;     // [G]

    // node pool [G*M]
    NodeKey* node_key;   // key + Ns, one 32-B record per node
    int32_t* node_turn;  // -1 = free (the node GC's scan reads this dense array)
    float* node_P;       // [G*M*AP]
    uint32_t* node_N;    // [G*M*AP]  bit31: Q is f32-typed
    float* node_Qf;      // [G*M*AP]  Q of f32-typed edges (N bit31 set): read with P and N
    double* node_Q;      // [G*M*AP]  Q of Python-float edges (bit31 clear): read only for those
    int32_t* free_stack; // [G*M]
    int32_t* free_top;   // [G]
    int32_t* live;       // [G] allocated nodes
    uint64_t* table;     // [G*H] (tag << 32) | (id + 1), 0 = empty

    // search path / leaf
    int32_t* path;       // [G*DMAX] (node << 10) | edge slot (compact, azg_kernels.hip edge_slots)
    int32_t* leaf_kind;  // [G]
    int32_t* leaf_depth; // [G]
    double* leaf_value;  // [G]
    uint64_t* leaf_own;
    uint64_t* leaf_opp;
    int32_t* leaf_turn;
    int32_t* leaf_cs;
    int32_t* leaf_slot;

    // per-move record
    int32_t* moves;      // [G]
    int64_t* game_id;    // [G]  global game index of the slot's game (seed = seed_base + game_id)
    int32_t* harvested;  // [G]  continuous batching: the finished game was handed off, slot idle
    int32_t* rec_action; // [G*max_moves]
    int8_t* rec_temp;    // [G*max_moves]
    int32_t* rec_counts; // [G*max_moves*A] or null

    // per-slot counters (no atomics: one wave per slot)
    int64_t* st_exp;
    int64_t* st_term;
    int64_t* st_fallback;
    int64_t* st_sims;
    int32_t* st_depth;
    int32_t* st_live_max;
    int32_t* err;        // [G] first error code seen in the slot
};

}  // namespace azg
