/*
 * yacht_hip.h - C ABI of libyacht_hip.so, the MI355X (gfx950) self-play engine for
 * Yacht Auction.  This is the drop-in boundary for the reference's hot path
 *   Coach.executeEpisode -> MCTS.getActionProb -> MCTS.search
 *     -> YachtGame.{getNextState,getValidMoves,getGameEnded,getCanonicalForm,...}
 *     -> NNetWrapper.predict
 * (paths relative to the reference repository iyioon/NYPC-Yacht-Auction).
 *
 * Conventions
 *  - Every array argument is a DEVICE pointer owned by the caller (hipMalloc /
 *    torch), unless the comment says "host".  `stream` is a hipStream_t (NULL = the
 *    default stream).  Calls are asynchronous on `stream` unless they say otherwise.
 *  - Return value: YK_OK (0) or a negative YK_ERR_* code (API / HIP / capacity error).
 *    The reference's per-call Python exceptions are reported per element in a
 *    `status` array (YK_ST_*), because a batch can contain both good and bad inputs.
 *  - A game state is the 64-byte packed yk_state_t (layout: DESIGN.md section 3; it is
 *    injective on exactly the fields of YachtGame.stringRepresentation, so two states
 *    are the same MCTS node iff their 8 words are equal).
 *  - Randomness: the reference draws from process-global numpy / `random` RNGs
 *    (YachtGame.py:154-159, MCTS.py:46, Coach.py:65).  Here every game owns a stream
 *    (seed, env_id, counter) of Philox4x32-10 draws; each die, tie-break, tie pick and
 *    sampling uniform consumes one counter value.  Given the same draws the results
 *    are identical to the reference (tests/test_oracle_golden.py, tests/test_gpu_*.py).
 *  - No torch types cross this boundary.
 */
#ifndef YACHT_HIP_H
#define YACHT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YK_ACTION_SIZE 3226   /* YachtGame.py:42 */
#define YK_NUM_BID_ACTIONS 202 /* YachtGame.py:32 */
#define YK_FEATURES 59        /* YachtGame.getBoardSize, NNet.py:47 */
#define YK_MASK_WORDS 101     /* ceil(3226 / 32) */

typedef struct { uint64_t w[8]; } yk_state_t;

/* return codes */
#define YK_OK 0
#define YK_ERR_ARG (-1)
#define YK_ERR_HIP (-2)
#define YK_ERR_NOMEM (-3)
#define YK_ERR_CAPACITY (-4) /* a fixed-size engine pool overflowed; results invalid */
#define YK_ERR_STATE (-5)    /* engine misuse (e.g. MCTS root round went backwards) */
#define YK_ERR_RANGE (-6)    /* a weight outside the fp16 split's range (|w| >= 65520: its hi plane overflows) */

/* per-element status of yk_step: the reference's exceptions */
#define YK_ST_OK 0
#define YK_ST_VALUE_BID 1   /* ValueError("Invalid action in BID phase")   YachtGame.py:268-269 */
#define YK_ST_VALUE_SCORE 2 /* ValueError("Invalid action in SCORE phase") YachtGame.py:306-307 */
#define YK_ST_RUNTIME 3     /* RuntimeError("Invalid phase/state")          YachtGame.py:372 */
#define YK_ST_ASSERT 4      /* AssertionError, _resolve_bids_and_assign     YachtGame.py:508 */
#define YK_ST_CAPACITY 5    /* a carry would exceed 10 dice (unreachable from getInitBoard) */

const char* yk_version(void);
/* last HIP error code seen by the library (hipError_t as int), 0 if none */
int yk_last_hip_error(void);
/* HOST: draw `ctr` of game `env`'s stream (Philox4x32-10, key = seed, counter = (ctr, env, 0)):
 * low 32 bits = word 0, high = word 1.  die = 1 + ((d >> 32) * 6 >> 32), below(n) likewise,
 * uniform = (d >> 11) * 2^-53. */
uint64_t yk_rng_draw64(uint64_t seed, uint32_t env, uint64_t ctr);

/* ---------------------------------------------------------------- Game plugin (batched)
 * Replaces YachtGame (yacht/YachtGame.py:210-467) behind Game.py:14-113.  Player values
 * follow the reference: 1 = player 1, anything else = player 2 (-1). */

/* getInitBoard (YachtGame.py:232-237): draws rollA then rollB (10 dice) from each game's
 * stream; rng_ctr[i] is read and advanced. */
int yk_init_board(yk_state_t* out, uint64_t* rng_ctr, const uint32_t* env_ids, uint64_t seed, int n,
                  void* stream);
/* getNextState (YachtGame.py:260-372, _resolve_bids_and_assign :502-542).  Pure: `in` is
 * not modified (out may alias in).  rng_ctr advanced by the draws made (tie-break, re-rolls).
 * status[i] != YK_ST_OK => out[i] / next_players[i] / rng_ctr[i] unspecified (the
 * reference raised).  The silent no-op of an illegal SCORE action is YK_ST_OK with the
 * state copied and the player flipped (YachtGame.py:312-314, 322-324). */
int yk_step(const yk_state_t* in, const int32_t* players, const int32_t* actions, uint64_t seed,
            const uint32_t* env_ids, uint64_t* rng_ctr, yk_state_t* out, int32_t* next_players, int8_t* status,
            int n, void* stream);
/* getValidMoves (YachtGame.py:374-406) as a bitmask: bit (a & 31) of mask[i*101 + a/32];
 * counts[i] = number of valid actions (may be NULL). */
int yk_valid_mask(const yk_state_t* in, const int32_t* players, uint32_t* mask, int32_t* counts, int n,
                  void* stream);
/* getGameEnded (YachtGame.py:408-428): result[i] in {0, 1e-4, 1, -1} (python float);
 * totals[i*2+{0,1}] = total_with_bonus of p1/p2 (YachtGame.py:128-130), may be NULL. */
int yk_ended(const yk_state_t* in, const int32_t* players, double* result, int32_t* totals, int n, void* stream);
/* getCanonicalForm (YachtGame.py:430-442): player 1 -> copy; else p1<->p2 and bids swapped
 * (the reference does NOT mask the pending bid, despite its docstring). */
int yk_canonical(const yk_state_t* in, const int32_t* players, yk_state_t* out, int n, void* stream);
/* score_category (YachtGame.py:57-108) of every (category, combo) on the mover's carry:
 * out[(i*12 + cat)*252 + combo]; -1 where combo position >= len(carry). */
int yk_score_table(const yk_state_t* in, const int32_t* players, int32_t* out, int n, void* stream);
/* score_category on explicit dice: dice[i*5..+5] in 1..6 -> out[i*12 + cat]. */
int yk_score_dice(const int8_t* dice, int32_t* out, int n, void* stream);
/* state_to_vec (yacht/NNet.py:65-86), bit-exact float32: x[i*59 + f]. */
int yk_featurize(const yk_state_t* in, float* x, int n, void* stream);
/* 64-bit transposition-key hash (stands in for stringRepresentation, YachtGame.py:448-467). */
int yk_key_hash(const yk_state_t* in, uint64_t* out, int n, void* stream);
/* GreedyYachtPlayer's heuristic (yacht/YachtPlayers.py:38-171) on canonical boards (device):
 * actions[i] = the heuristic's action, or -1 when it is not a valid move (the player then
 * plays np.random.choice(legal), YachtPlayers.py:199-214). */
int yk_greedy_action(const yk_state_t* states, int32_t* actions, int n, void* stream);
/* Deterministic test prior (oracle/spec.py hash_prior): pi[i*3226 + a], v[i]. */
int yk_hash_prior(const yk_state_t* in, float* pi, float* v, int n, void* stream);

/* ---------------------------------------------------------------- NeuralNet.predict
 * Replaces NNetWrapper.predict (yacht/NNet.py:177-195) over YachtNNet
 * (yacht/pytorch/YachtNNet.py:8-70), eval mode, batched, float32 (MFMA f32). */
typedef struct yk_net yk_net_t;
/* params: HOST float32 arrays in YachtNNet.state_dict() order (inp.0.weight, inp.0.bias,
 * inp.1.weight, inp.1.bias, blocks.{b}.{fc1,ln1,fc2,ln2}.{weight,bias}, pi_head.0.*,
 * pi_head.2.*, v_head.0.*, v_head.2.*, v_head.4.*).  hidden in {64,128,256,512}, nblocks 0-64.
 * YK_ERR_RANGE when a finite weight of a Linear layer overflows the fp16 hi plane of the
 * f32-equivalent split (|w| >= 65520): the planes would hold inf where torch holds a number. */
int yk_net_create(yk_net_t** net, int hidden, int nblocks, const float* const* params, int nparams);
/* pi[i*3226 + a] = exp(log_softmax(logits)), v[i] = tanh(v_head). */
int yk_net_predict(yk_net_t* net, const yk_state_t* states, float* pi, float* v, int n, void* stream);
/* same from explicit feature rows x[i*59 + f] */
int yk_net_predict_features(yk_net_t* net, const float* x, float* pi, float* v, int n, void* stream);
/* The prior the self-play engine expands a leaf with (MCTS.py:86-88 inside yk_selfplay), before
 * its renormalisation: pi[i*3226 + a] = exp(x_a - m - l) at the valid actions of canonical state
 * i (getValidMoves(s, 1)), 0 elsewhere, with (m, l) the softmax statistics over the actions of the
 * 16-action tiles holding those valid actions - or over all 3226 logits (NNetWrapper.predict's pi,
 * masked) when a weight-norm bound cannot rule out that every valid pi underflows in the full
 * softmax.  Renormalised over the valid actions it is MCTS.py:88-91's P either way. */
int yk_net_leaf_prior(yk_net_t* net, const yk_state_t* states, float* pi, float* v, int n, void* stream);
/* The submission bot's move (replaces AIPlayer.get_move's network part,
 * yacht/submission/agent.py:248-280): for canonical states (the mover is p1), the action of
 * highest softmax probability among the decodable ones (agent.py:150-187, the same set as
 * getValidMoves), lowest index on equal probability; -1 when none.  probs (optional) gets
 * that probability.  Device pointers. */
int yk_net_policy_action(yk_net_t* net, const yk_state_t* states, int32_t* actions, float* probs, int n,
                         void* stream);
int yk_net_destroy(yk_net_t* net);
/* Device-side check flags of this net's forwards since the last call (cleared by it; synchronises
 * the device): YK_NET_ERR_SYNC - a wave of the value head timed out waiting for v_head.2's columns
 * (its v row is then not trustworthy).  0 when every forward completed its hand-offs. */
#define YK_NET_ERR_SYNC 1u
int yk_net_errors(yk_net_t* net, uint32_t* flags);
/* Precision of every forward of this net (predict, leaf prior, the engine's expansions):
 * YK_PREDICT_F32 (default) - f32-equivalent products (fp16 hi/lo planes, three MFMAs each; within
 * 1e-5 of the reference's float32 CPU path); YK_PREDICT_F16 - fp16 weights and GEMM inputs with
 * f32 accumulation, one MFMA per product: the operand precision of the reference's own GPU
 * predict under autocast('cuda') (yacht/NNet.py:186-189), but with f32 outputs - the Linear
 * outputs and bias adds stay f32 where autocast rounds them to fp16, so it is closer to float32
 * than autocast is and not bit-equal to it.  LayerNorm, SiLU, softmax and tanh stay f32. */
#define YK_PREDICT_F32 0
#define YK_PREDICT_F16 1
int yk_net_set_precision(yk_net_t* net, int mode);

/* ---------------------------------------------------------------- self-play engine
 * Batched Coach.executeEpisode (Coach.py:34-72) over n_envs games in lock-step; every game
 * runs MCTS.getActionProb (MCTS.py:28-54) / MCTS.search (MCTS.py:56-164) with its own
 * tree (reset per episode, Coach.py:93). */
typedef struct {
    int n_envs;             /* games per batch (per GPU) */
    int sims;               /* numMCTSSims */
    double cpuct;           /* cpuct */
    int temp_threshold;     /* tempThreshold */
    int max_moves;          /* record capacity per game (every real game has 48 moves) */
    int prior;              /* 0 = yk_net (MLP), 1 = hash prior (test) */
    int record_predictions; /* test: keep every expansion's (Ps * valids, v, leaf) of sampled games */
    int max_expansions;     /* capacity of that record per game (record_predictions only) */
    int64_t arena_entries;  /* per game per generation P/edge-slot entries; 0 = default */
    int record_stride;      /* record_predictions samples games e with e % record_stride == 0 (0 = 1:
                               every game); recording never changes the search path */
    int groups;             /* game groups, each on its own stream so that one group's forward runs
                               beside another's expand (results do not depend on it); 0 = auto
                               (2 with the net prior at >= 8192 games, else 1), at most 8 */
    int dual_trees;         /* arena: two trees per game, so MCTS vs MCTS plays two MCTS objects with
                               their own trees and nets (Coach.py:117-125's pmcts / nmcts) */
} yk_engine_config_t;

typedef struct yk_engine yk_engine_t;
int yk_engine_create(yk_engine_t** eng, const yk_engine_config_t* cfg, yk_net_t* net);
int yk_engine_destroy(yk_engine_t* eng);
/* Plays one complete episode for each of the n_envs games (game i uses stream env_base+i).
 * Synchronises `stream` once per real move to test termination.  Returns YK_OK, or
 * YK_ERR_CAPACITY / YK_ERR_STATE if a device-side check failed (see yk_engine_stats). */
int yk_selfplay(yk_engine_t* eng, uint64_t seed, uint32_t env_base, void* stream);
/* Per-kernel timing with HIP events on the engine's stream; resets the accumulators.
 * enable = 0 off, k > 0 on: the per-move launches are timed every time, the per-simulation
 * forward / expand pair in every k-th simulation of a move (1 = all; an event record between
 * dependent launches costs GPU time, so a stride keeps the timed batch's rate).
 * yk_engine_kernel_times (launches counts the timed ones): HOST ms[8],
 * launches[8] for classes 0 first descent of a move, 1 forward (the whole predict), 2 unused,
 * 3 expand + backup + the next descent, 4 move begin (root / tree compaction), 5 move end
 * (policy, sampling, real step). */
int yk_engine_profile(yk_engine_t* eng, int enable);
int yk_engine_kernel_times(yk_engine_t* eng, double* ms, int64_t* launches);
/* HOST out[16]: 0 expansions, 1 valid entries scanned by UCB, 2 real moves (max over games),
 * 3 device error flags, 4 max live nodes, 5 max live edges, 6 max arena entries used (per shard),
 * 7 new-node valid entries written, 8 search path edges backed up, 9 lock-step sims run,
 * 10-13 node / edge / arena / visit capacities, 14 game groups, 15 forward head parts (workgroups per 16-row tile) */
int yk_engine_stats(yk_engine_t* eng, int64_t* out);
/* Further counters of the last batch, summed over games; writes out[0 .. n-1] of:
 * 0 edges gathered by the UCB scans (one 16-B edge per visited entry scanned, MCTS.py:122-133; with
 *   stats 1 and 7-8 the expand's algorithmic bytes, bench.py roofline_env) */
int yk_engine_counters(yk_engine_t* eng, int64_t* out, int n);
/* Copies the last episode batch to HOST arrays (any may be NULL):
 *   states[n][max_moves][8]  canonical board of each example (Coach.py:57,61)
 *   info[n][max_moves][8]    temp, player, action, expansions-so-far, root Ns, n visited, status, 0
 *   ctr[n][max_moves][2]     stream counter before the search / before the real step
 *   values[n][max_moves]     example value r*(-1)**(player != curPlayer) (Coach.py:72)
 *   final_states[n][8], n_moves[n]
 *   visits_off[n*max_moves+1], visits[...][2] (action, N): root visit counts, ascending
 *   action (size: yk_engine_records(...) with visits=NULL returns the total in *n_visits). */
int yk_engine_records(yk_engine_t* eng, uint64_t* states, int32_t* info, uint64_t* ctr, double* values,
                      uint64_t* final_states, int32_t* n_moves, int64_t* visits_off, int32_t* visits,
                      int64_t* n_visits);
/* record_predictions, for the R = ceil(n_envs / record_stride) sampled games (game r * record_stride):
 * HOST pi[R][max_expansions][3226] = the prior each expansion was made with, masked (MCTS.py:86-88:
 * Ps * valids, before the renormalisation, the production valid-only softmax of yk_net_leaf_prior),
 * v[R][max_expansions], leaves[R][max_expansions] the expanded canonical states, count[R] the
 * expansions of each game (> max_expansions: the record was truncated).  Any may be NULL. */
int yk_engine_predictions(yk_engine_t* eng, float* pi, float* v, yk_state_t* leaves, int32_t* count);
/* Fixed-size trajectory records of the last batch for the multi-GPU all-gather:
 * yk_engine_record_bytes = size of the packed image; yk_engine_pack_records copies it
 * (device to device, async on `stream`) into dst (device, >= that many bytes).  Image:
 * states[n][M][8] u64 | info[n][M][8] i32 | ctr[n][M][2] u64 | values[n][M] f64 |
 * visits[n][VCAP] u32 (action << 16 | N) | visits_off[n][M+1] i32 | n_moves[n] i32 |
 * final_states[n][8] u64 (M = max_moves, VCAP = 2 * M * max(sims, 32)). */
int64_t yk_engine_record_bytes(yk_engine_t* eng);
int yk_engine_pack_records(yk_engine_t* eng, void* dst, int64_t capacity, void* stream);

/* The replay buffer's examples: n_images packed record images back to back (each
 * yk_engine_record_bytes of an engine with n_envs games, max_moves, sims - e.g. every rank's image
 * after the all-gather) -> one example per move of the first n_games games (image-major; < 0 = all),
 * in (image, game, move) order: Coach.executeEpisode's (canonicalBoard, pi, v) (Coach.py:57-72)
 * as NNetWrapper.train consumes it - states[k] the board, targets[k] = argmax(pi) (NNet.py:145-146:
 * the played action at temp 0, the most visited action at temp 1, lowest on ties), values[k] = v
 * (float32).  The first `skip` examples are dropped (the maxlenOfQueue deque keeps the last ones,
 * Coach.py:86-90); at most `capacity` are written.  states = NULL: count only.  HOST *n_examples =
 * examples written (or countable).  Synchronises `stream`. */
int yk_examples_from_records(const void* images, int n_images, int n_envs, int max_moves, int sims,
                             int64_t n_games, int64_t skip, int64_t capacity, yk_state_t* states, int32_t* targets,
                             float* values, int64_t* n_examples, void* stream);
/* The full policies of the same examples (Coach.py:57-61: MCTS.getActionProb's pi, MCTS.py:44-54 -
 * one-hot at the played action at temp 0, N / sum N at temp 1) as a sparse CSR of their nonzero
 * entries, for the examples file (Coach.py:144-151) and code that iterates the reference's tuples.
 * Examples skip .. skip + n_examples - 1 (as yk_examples_from_records numbers them; n_examples <=
 * the examples after skip).  DEVICE pi_indptr[n_examples + 1] (always written: example k's entries
 * are pi_indptr[k] .. pi_indptr[k+1]-1), pi_cols[nnz] (actions, ascending), pi_vals[nnz] (float64),
 * values[n_examples] (float64 v, may be NULL).  pi_cols = NULL: count only.  HOST *nnz = the
 * entries (YK_ERR_CAPACITY if more than nnz_capacity).  Synchronises `stream`. */
int yk_examples_policies(const void* images, int n_images, int n_envs, int max_moves, int sims, int64_t n_games,
                         int64_t skip, int64_t n_examples, int64_t* pi_indptr, int32_t* pi_cols, double* pi_vals,
                         int64_t nnz_capacity, double* values, int64_t* nnz, void* stream);

/* ---------------------------------------------------------------- Arena
 * Batched Arena.playGame (Arena.py:30-93), n_envs games in lock-step: `agent` in seat
 * agent_seat[i] (HOST, [n]; 1 = moves first, -1) against `opponent` in the other seat, each a
 * YK_PLAYER_*: MCTS = np.argmax(MCTS.getActionProb(board, temp=0)) (Coach.py:124-125) with the
 * engine's net / prior and sims, one tree per game for the whole game; RANDOM =
 * RandomYachtPlayer (YachtPlayers.py:174-183); GREEDY = GreedyYachtPlayer (:186-214).  Game i
 * uses stream env_base+i for every draw.  Returns like yk_selfplay. */
#define YK_PLAYER_MCTS 0
#define YK_PLAYER_RANDOM 1
#define YK_PLAYER_GREEDY 2
int yk_arena(yk_engine_t* eng, uint64_t seed, uint32_t env_base, const int32_t* agent_seat, int agent, int opponent,
             void* stream);
/* HOST outputs of the last yk_arena (any may be NULL): result[n] = curPlayer * getGameEnded
 * (Arena.py:93, from player 1's view: +1 / -1 / +-1e-4 draw), totals[n][2] (player 1, player 2,
 * with bonus), n_moves[n], actions[n][max_moves] (-1 past the end), final_states[n][8],
 * rng_ctr[n] (stream counter at the end).  yk_engine_records also works after yk_arena. */
/* The opponent seat's net for MCTS vs MCTS arenas of a dual_trees engine (default: the engine's
 * net).  The gating arena of Coach.learn: yk_arena(agent = previous net's MCTS, opponent = new). */
int yk_engine_set_opponent_net(yk_engine_t* eng, yk_net_t* net);
int yk_arena_results(yk_engine_t* eng, double* result, int32_t* totals, int32_t* n_moves, int32_t* actions,
                     uint64_t* final_states, uint64_t* rng_ctr);

/* ---------------------------------------------------------------- MCTS plugin
 * MCTS(game, nnet, args).getActionProb (MCTS.py:28-54) for n_envs independent searches
 * sharing nothing: runs `sims` searches from roots[i] (device, canonical boards) with
 * persistent trees, drawing from game i's stream (rng_ctr[i], advanced), and writes the
 * root visit counts counts[i*3226 + a] (device).  Roots must not go back in round
 * (trees keep only nodes of rounds >= the root's, which is parity-safe because a game's
 * round never decreases).  yk_mcts_reset clears all trees. */
int yk_mcts_search(yk_engine_t* eng, const yk_state_t* roots, uint64_t seed, const uint32_t* env_ids,
                   uint64_t* rng_ctr, int sims, int32_t* counts, void* stream);
int yk_mcts_reset(yk_engine_t* eng);

/* ---------------------------------------------------------------- training
 * NNetWrapper.train (yacht/NNet.py:118-174): one optimiser step per minibatch of YachtNNet -
 * loss = cross_entropy(logits, argmax(pi)) + vloss_weight * mse(v, z) (:143-148),
 * clip_grad_norm_(max_grad_norm) (:152-153), AdamW(lr, weight_decay) (:109-110).  Two modes:
 * amp = 0, float32 (the reference's CPU path, :157-165); amp = 1, the reference's GPU path
 * (:113-116, 141-155): autocast('cuda') arithmetic (fp16 Linear layers with f32 accumulation,
 * f32 LayerNorm and losses) on fp16 MFMA kernels, loss scaling with GradScaler('cuda')
 * semantics (init_scale, x2 after growth_interval finite steps, x0.5 and the step skipped on an
 * inf / nan gradient), unscale before the clip.  Dropout masks come from the Philox stream
 * (seed, layer, step, row, column), not torch's generator; rows are numbered from the offset set
 * by yk_trainer_set_row_offset (0 by default; it applies to the next backward only and resets to 0
 * after it), so ranks splitting one minibatch draw the masks of the whole minibatch.  Parameters, gradients and Adam moments are flat device buffers in
 * state_dict order. */
typedef struct {
    int max_batch;          /* batch_size (rows per step, upper bound) */
    float lr, weight_decay; /* AdamW */
    float beta1, beta2, eps;
    float max_grad_norm;    /* 5.0 in the reference */
    float vloss_weight;     /* 1.5 in main.py */
    float dropout;          /* 0.3 in main.py; 0 for deterministic parity tests */
    uint64_t seed;          /* dropout stream */
    int amp;                /* 0: float32 step; 1: mixed precision (autocast + GradScaler) */
    float init_scale;       /* GradScaler init_scale (0: 65536) */
    int growth_interval;    /* GradScaler growth_interval (0: 2000) */
} yk_train_config_t;
typedef struct yk_trainer yk_trainer_t;
/* params: HOST float32 arrays in YachtNNet.state_dict() order (as yk_net_create) */
int yk_trainer_create(yk_trainer_t** t, int hidden, int nblocks, const float* const* params, int nparams,
                      const yk_train_config_t* cfg);
int yk_trainer_destroy(yk_trainer_t* t);
/* device pointers of the flat parameter and gradient buffers (for a DDP all-reduce of grads) */
int yk_trainer_buffers(yk_trainer_t* t, float** params, float** grads, int64_t* nparams);
/* forward + backward of one minibatch into the gradient buffer (overwritten).  Example i of the
 * batch is replay entry batch_idx[i] (device, or NULL for 0..batch-1): states[] packed canonical
 * boards, targets[] = argmax(pi) (NNet.py:145-146), values[] = v.  Losses: yk_trainer_losses. */
int yk_trainer_backward(yk_trainer_t* t, const yk_state_t* states, const int32_t* targets, const float* values,
                        const int32_t* batch_idx, int batch, void* stream);
/* clip_grad_norm_ + AdamW on the (possibly all-reduced) gradient buffer; advances the step */
int yk_trainer_apply(yk_trainer_t* t, void* stream);
/* yk_trainer_backward + yk_trainer_apply; in amp mode the gradient launches also sum the unscaled
 * grad norm (nothing can change the buffer between the two), so apply does not re-read it */
int yk_trainer_step(yk_trainer_t* t, const yk_state_t* states, const int32_t* targets, const float* values,
                    const int32_t* batch_idx, int batch, void* stream);
/* HOST out[3]: sum over the last batch of cross-entropy, of squared value error; grad sq-norm */
int yk_trainer_losses(yk_trainer_t* t, double* out);
/* a reporting epoch's "Avg Loss" (NNet.py:150-160) without a host round trip per minibatch:
 * begin zeroes a device accumulator; every later yk_trainer_backward adds its batch's
 * ce/b + vloss_weight*se/b to it (one 1-thread launch on that stream) until end, which
 * synchronises and writes HOST out[2] = (sum of those batch losses, batches) */
int yk_trainer_epoch_loss_begin(yk_trainer_t* t, double vloss_weight);
int yk_trainer_epoch_loss_end(yk_trainer_t* t, double* out);
/* copy parameters (which 0), gradients (1), exp_avg (2), exp_avg_sq (3) to / from HOST arrays in
 * state_dict order (NULL entries skipped); set: step >= 0 also sets the optimiser step count */
int yk_trainer_get(yk_trainer_t* t, int which, float* const* out);
int yk_trainer_set(yk_trainer_t* t, int which, const float* const* in, int64_t step);
int64_t yk_trainer_step_count(yk_trainer_t* t);
/* the global row number of the next backward's first example (dropout masks; DDP ranks pass
 * their offset into the minibatch) */
int yk_trainer_set_row_offset(yk_trainer_t* t, int64_t row0);
/* HOST out[4] (amp mode): loss scale, growth tracker, optimiser steps taken, last step skipped */
int yk_trainer_amp_state(yk_trainer_t* t, double* out);

#ifdef __cplusplus
}
#endif
#endif /* YACHT_HIP_H */
