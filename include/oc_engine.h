/*
 * oc_engine.h -- C-ABI of the MI355X batched Overcooked step engine (liboc_engine.so).
 *
 * The reference (deletfsi/gym-cooking) is pure Python and has no FFI; each entry point
 * below replaces one reference routine on the environment-step hot path and is what a
 * ctypes/cffi binding of that routine binds (INTEGRATION.md shows the binding):
 *
 *   oc_create / oc_destroy   <- OvercookedEnvironment.load_level + run_recipes
 *                               (gym_cooking/envs/overcooked_environment.py:130-198, :396-473)
 *   oc_reset                 <- OvercookedEnvironment.reset      (overcooked_environment.py:201-250)
 *   oc_step, oc_step_n       <- OvercookedEnvironment.step       (overcooked_environment.py:255-306)
 *                               = check_collisions (:724-762) + execute_navigation/interact
 *                               (:767-770, gym_cooking/utils/interact.py:4-89) + done/reward (:316-376)
 *   oc_gen_actions           <- synthetic action streams (the reference env has no RNG)
 *   oc_stats_*               <- the per-episode bookkeeping main.py keeps in its metrics Bag
 *                               (gym_cooking/misc/metrics/metrics_bag.py:40-72), reduced per GPU
 *
 * Conventions
 *  - All entry points return 0 on success and a negative OC_E* code on failure; the message
 *    of the last failure on the calling thread is available from oc_last_error(), and the
 *    last failure of a call on a given handle from oc_get_last_error(h, buf, size).
 *  - Every buffer is caller-owned device memory (e.g. torch ROCm tensors); the engine never
 *    allocates in oc_step / oc_reset / oc_gen_actions, so they are hipGraph-capturable.
 *  - `stream` is a hipStream_t passed as void* (NULL = the null stream).  Calls are
 *    stream-ordered and not synchronised; a handle is not thread-safe.
 *  - State is structure-of-arrays: `num_planes` byte planes of `pitch` bytes each (see
 *    oc_layout).  Env e of plane p lives at byte p*pitch + e (the t plane holds u16 at
 *    2*e and spans two planes).  pitch = B rounded up to OC_PITCH_ALIGN.
 *  - Columns [B, pitch) of an output plane belong to the engine: the step kernels move four
 *    envs per 32-bit word, so the columns of the batch's last word past B may be rewritten
 *    (the state planes with what the input held there or its step, exec_actions / coll_mask
 *    with no-op / 0).  Nothing at or past the next multiple of 4 above B is written, and no
 *    statistic counts a column past B.
 */
#ifndef OC_ENGINE_H_
#define OC_ENGINE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OC_ABI_VERSION 10

#define OC_MAX_AGENTS 4
#define OC_MAX_ITEMS 16  /* item slots: K = 4, 8 or 16 per level */
#define OC_MAX_CELLS 1024       /* grid cells (width and height <= 255 each) */
#define OC_MAX_NARROW_CELLS 255 /* levels of at most this many cells have byte cell ids (0xFF is
                                   OC_LOC_DEAD); larger ("wide") levels u16 ids (OC_LOC_DEAD16) */
#define OC_MAX_GOALS 4
#define OC_PITCH_ALIGN 4096

/* status codes */
#define OC_OK 0
#define OC_EINVAL (-1)   /* bad argument / unsupported shape */
#define OC_EHIP (-2)     /* HIP runtime error */
#define OC_ELEVEL (-3)   /* level outside the exact-semantics envelope */

/* tile classes (gym_cooking/utils/core.py:28-120; only Floor is non-collidable) */
#define OC_TILE_FLOOR 0
#define OC_TILE_COUNTER 1
#define OC_TILE_CUTBOARD 2
#define OC_TILE_DELIVERY 3

/* Item content masks, two encodings (oc_level_desc.encoding).
 * OC_ENC_PRESENCE: presence T,L,O,P + chopped T,L,O; exact for levels with at
 *   most one of each food type (every shipped level).
 * OC_ENC_COUNTS: the multiset of a core.Object's contents (equality is by full_name, a sorted
 *   multiset: gym_cooking/utils/core.py:143-171): a 2-bit count per food, a plate bit and a
 *   Fresh bit.  Exact for levels with up to 3 of each food type (load_level makes one Object
 *   per map character with no uniqueness check, overcooked_environment.py:158-165): an object
 *   of more than one content is a merge, and mergeable() (core.py:222-241) admits only foods
 *   in their last state and at most one plate, so a merged object is all-Chopped and the
 *   Fresh bit only ever marks a single fresh food.  Goal masks never carry it. */
#define OC_M_TOMATO 0x01u
#define OC_M_LETTUCE 0x02u
#define OC_M_ONION 0x04u
#define OC_M_PLATE 0x08u
#define OC_M_CHOPPED_SHIFT 4
#define OC_ENC_PRESENCE 0
#define OC_ENC_COUNTS 1
#define OC_MC_TOMATO 0x01u   /* count field bits 0-1 */
#define OC_MC_LETTUCE 0x04u  /* bits 2-3 */
#define OC_MC_ONION 0x10u    /* bits 4-5 */
#define OC_MC_PLATE 0x40u
#define OC_MC_FRESH 0x80u    /* a single food in its Fresh state */
#define OC_MC_MAX_PER_FOOD 3

/* action codes: World.NAV_ACTIONS order (gym_cooking/utils/world.py:16) + no-op.
 * Codes > 4 are treated as OC_ACT_NOOP. */
#define OC_ACT_DOWN 0   /* ( 0, 1) */
#define OC_ACT_UP 1     /* ( 0,-1) */
#define OC_ACT_LEFT 2   /* (-1, 0) */
#define OC_ACT_RIGHT 3  /* ( 1, 0) */
#define OC_ACT_NOOP 4   /* ( 0, 0) */

#define OC_HOLD_NONE 0xFFu
#define OC_LOC_DEAD 0xFFu
#define OC_LOC_DEAD16 0xFFFFu

/* flags plane bits */
#define OC_FLAG_DONE 0x01u    /* done() returned True (overcooked_environment.py:316-363) */
#define OC_FLAG_SUCCESS 0x02u /* reward() == 1 (overcooked_environment.py:365-376) */
#define OC_FLAG_ERR 0x04u     /* the reference's step raises: at new_obs = copy.copy(self)
                                 (overcooked_environment.py:289 -> world.py:417) when two
                                 co-located agents both hold, or, on a level with a Floor on its
                                 border and two or more agents, in check_collisions when an action
                                 points off the grid (is_collision :692-700 -> get_gridsquare_at
                                 asserts, world.py:429; the state is then unchanged but t, the
                                 executed actions no-ops).  ERR implies DONE. */

/* per-GPU episode statistics (oc_stats_reduce output, uint64 each) */
#define OC_STAT_EPISODES 0   /* envs whose episode ended this window (DONE newly set) */
#define OC_STAT_SUCCESSES 1  /* of those, reward 1 */
#define OC_STAT_STEPS 2      /* sum of t over ended episodes (episode lengths) */
#define OC_STAT_COLLISIONS 3 /* sum over steps of colliding agent pairs (CollisionRepr count) */
#define OC_STAT_ERRORS 4     /* envs that hit the ERR condition */
#define OC_NSTATS 5

typedef struct oc_level_desc {
    int32_t width, height;           /* 3..255; width*height <= OC_MAX_CELLS */
    int32_t num_items;               /* <= OC_MAX_ITEMS; OC_ENC_PRESENCE: at most one of each food
                                        type, OC_ENC_COUNTS: at most OC_MC_MAX_PER_FOOD */
    int32_t num_spawns;              /* >= num_agents */
    int32_t num_goals;               /* 1..OC_MAX_GOALS Deliver goal masks */
    uint8_t tiles[OC_MAX_CELLS];     /* OC_TILE_* per cell, cell = y*width + x */
    uint16_t item_cell[OC_MAX_ITEMS]; /* initial item cells, map scan order */
    uint8_t item_mask[OC_MAX_ITEMS]; /* initial item content masks */
    uint8_t spawn_x[OC_MAX_AGENTS];
    uint8_t spawn_y[OC_MAX_AGENTS];
    uint8_t goal_mask[OC_MAX_GOALS];
    int32_t encoding;                /* OC_ENC_*: how item_mask / goal_mask (and every state's item
                                        masks and oc_subtask masks) encode contents */
} oc_level_desc;

typedef struct oc_layout {
    int64_t pitch;          /* bytes per byte-plane */
    int64_t state_bytes;    /* num_planes * pitch */
    int32_t num_agents;     /* A */
    int32_t num_items;      /* K (item slots; >= level items, extra slots dead) */
    int32_t plane_agent_x;  /* A planes, u8 */
    int32_t plane_agent_y;  /* A planes, u8 */
    int32_t plane_agent_hold; /* A planes, u8 item slot or OC_HOLD_NONE */
    int32_t plane_item_loc; /* K planes: the item cells (u8, OC_LOC_DEAD = none), or on a wide level
                               their low bytes */
    int32_t plane_item_mask;/* K planes, u8 content mask */
    int32_t plane_t;        /* u16 step counter, spans 2 planes */
    int32_t plane_flags;    /* u8 OC_FLAG_* */
    int32_t num_planes;     /* 3A + 2K + 3; wide: 3A + 3K + 3 */
    int32_t plane_item_loc_hi; /* wide levels: K planes, the item cells' high bytes (cell =
                                  lo | hi << 8, OC_LOC_DEAD16 = none); -1 on a narrow level */
    int32_t cell_bytes;     /* 1 (narrow) or 2 (wide: more than OC_MAX_NARROW_CELLS cells) */
} oc_layout;

typedef struct oc_handle oc_handle;

/* Library identity. */
int oc_abi_version(void);
const char* oc_last_error(void);

/* The message of the last failed call on handle h (the same text oc_last_error() gave the
 * calling thread then), copied NUL-terminated into buf (at most size bytes); "" when no call
 * on h has failed.  Returns the message length. */
int oc_get_last_error(const oc_handle* h, char* buf, int64_t size);

/* Static level tables + episode settings.  max_T = --max-num-timesteps (main.py:24), 0 to
 * 65,535 (the u16 step counter; round 4 refused past 32,767); 0 = no limit, where the counter
 * wraps after 65,535 steps (the reference's keeps counting; nothing else reads it).  device = HIP ordinal the handle's launches target (recorded, validated), or
 * OC_DEVICE_HOST: a host-only handle that makes no HIP call at all (no device query, no
 * device tables); only the host entry points (oc_get_layout, oc_cpu_step, oc_reachability,
 * oc_stats_size) take it, the device ones return OC_EINVAL. */
#define OC_DEVICE_HOST (-1)
int oc_create(const oc_level_desc* level, int32_t num_agents, int32_t max_T, int32_t device,
              oc_handle** out);
int oc_destroy(oc_handle* h);

/* Layout of a B-env batch for this handle. */
int oc_get_layout(const oc_handle* h, int64_t B, oc_layout* out);

/* Broadcast the level's initial state (reset(), overcooked_environment.py:201-250) to B envs. */
int oc_reset(const oc_handle* h, void* state, int64_t B, void* stream);

/* One env step for B envs (step(), overcooked_environment.py:255-306).
 *   state_in/state_out : layout buffers (may alias: in-place is allowed)
 *   actions            : u8 [A][pitch] action codes
 *   exec_actions       : u8 [A][pitch] executed (post-collision) codes = env.agent_actions
 *                        (overcooked_environment.py:770); nullable
 *   coll_mask          : u8 [pitch] colliding pairs in itertools.combinations order
 *                        (0,1),(0,2),(0,3),(1,2),(1,3),(2,3) (overcooked_environment.py:731-752); nullable
 *   stats              : u64 partial-sum buffer of oc_stats_size() bytes (zeroed by the caller
 *                        once per window); nullable
 * An env whose input flags carry OC_FLAG_DONE is reset to the level template instead of
 * stepped (next-step auto-reset; its exec actions read OC_ACT_NOOP, coll 0). */
int oc_step(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions,
            uint8_t* exec_actions, uint8_t* coll_mask, uint64_t* stats, int64_t B, void* stream);

/* n consecutive steps in one launch, identical to n oc_step calls with ping-pong buffers
 * (state_in -> state_out after n steps).  The state stays in registers between steps, so the
 * state is read from HBM once per launch instead of once per step.
 *   actions      : n x u8 [A][pitch], step r at actions + r*A*pitch
 *   traj         : nullable; n x [num_planes][pitch]: the state after every step (traj[r] equals
 *                  the state_out of the r-th oc_step).  state_in must lie outside it; state_out
 *                  may be exactly its last state, traj + (n-1)*num_planes*pitch, which is then
 *                  written once (no second copy of the final state); any other overlap is refused
 *   exec_actions : nullable; n x u8 [A][pitch];  coll_mask : nullable; n x u8 [pitch]
 *   stats        : accumulated over the n steps (the oc_step layout, plus completion counters
 *                  after the statistics rows that must be zero when a launch with totals starts:
 *                  a zeroed buffer from the caller, which every completed launch leaves zeroed);
 *                  nullable.  Concurrent oc_step_n calls with totals (different streams) must
 *                  not share a stats buffer, and a buffer whose launch faulted must be re-zeroed
 *   totals       : nullable (needs stats); OC_NSTATS device uint64: the launch's last wave
 *                  folds the stats buffer into it, i.e. oc_stats_reduce after the steps
 *                  without a second launch (main.py's per-episode bookkeeping for the window).
 * A call longer than one launch can carry (the trajectory and action offsets of a launch stay
 * < 2 GiB, and at most 4096 steps) runs as several launches, each starting from the previous
 * one's last trajectory state; the results are the same. */
int oc_step_n(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions, void* traj,
              uint8_t* exec_actions, uint8_t* coll_mask, uint64_t* stats, uint64_t* totals, int64_t B, int32_t n,
              void* stream);

/* The same step on the host, for a caller without a GPU (a CPU restatement behind
 * the same ABI, same layout).  step(), overcooked_environment.py:255-306, exactly as oc_step:
 * the host pass of the kernel's own SWAR step (oc_swar.h, four envs per 32-bit word, the
 * v_perm / v_bitop3 byte operations restated bit for bit), threaded over env ranges.
 *   state_in/state_out, actions, exec_actions, coll_mask : HOST buffers in the oc_step layout
 *                 (state_in may equal state_out)
 *   totals      : nullable; OC_NSTATS host uint64, the window's statistics ADDED to it
 *   nthreads    : worker threads (0 = the host's hardware threads; at least 16 Ki envs each)
 * It never touches the device; oc_step / oc_step_n never call it (no CPU fallback). */
int oc_cpu_step(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions,
                uint8_t* exec_actions, uint8_t* coll_mask, uint64_t* totals, int64_t B, int32_t nthreads);

/* Synthetic i.i.d. uniform action codes 0..4 for B envs at step `step`:
 * code = splitmix64(seed ^ gid*0x9E3779B97F4A7C15 ^ step*0xC2B2AE3D27D4EB4F ^ agent) % 5,
 * gid = env_offset + e (global env id: identical for any GPU count). */
int oc_gen_actions(const oc_handle* h, uint8_t* actions, int64_t B, int64_t env_offset,
                   int64_t step, uint64_t seed, void* stream);

/* Order-sensitive 64-bit checksum of the state of envs [0, B) into *out (device uint64):
 *   sum_e (2e+1) * sum_p (byte_p(e) + 1) * 0x9E3779B97F4A7C15 * (2p+1)   (mod 2^64),
 * p over the byte planes (t as its low/high byte).  A size-independent parity probe for full
 * batches (compare with a host computation without copying the batch back). */
int oc_state_checksum(const oc_handle* h, const void* state, int64_t B, uint64_t* out, void* stream);

/* Statistics: size of the partial buffer for B envs, and its reduction into OC_NSTATS
 * device uint64 totals. */
int oc_stats_size(const oc_handle* h, int64_t B, int64_t* nbytes);
int oc_stats_reduce(const oc_handle* h, const uint64_t* stats, int64_t B, uint64_t* totals,
                    void* stream);

/* ---------------------------------------------------------------------------------------
 * Navigation-planner rollout: what E2E_BRTDP evaluates per (state,
 * subtask allocation, action).  Replaces, per row:
 *   _configure_planner_level, Level 0   navigation_planner/planners/e2e_brtdp.py:383-406
 *     (agents outside the subtask become collidable AgentCounters, utils/core.py:79-93,
 *      and the items they hold leave the world)
 *   get_actions / get_single_actions    e2e_brtdp.py:151-206, navigation_planner/utils.py:55-90
 *   T(state_repr, action)               e2e_brtdp.py:103-149 (interact per subtask agent in
 *                                       order, no collision pass, joint co-location assert)
 *   is_goal_state                       e2e_brtdp.py:435-566
 *   get_lower_bound_for_subtask_given_objs  gym_cooking/envs/overcooked_environment.py:480-664
 *     -> World.get_lower_bound_between(_helper), check_bound   gym_cooking/utils/world.py:115-283
 *     over the static reachability graph            world.py:67-108 (BFS table built in oc_create)
 * ------------------------------------------------------------------------------------- */
#define OC_MAX_SUBTASKS 64
#define OC_SUB_NONE 0    /* subtask None: every state is a goal state */
#define OC_SUB_CHOP 1    /* Chop(food)     gym_cooking/recipe_planner/utils.py:128 */
#define OC_SUB_MERGE 2   /* Merge(a, b)    recipe_planner/utils.py:142 */
#define OC_SUB_DELIVER 3 /* Deliver(dish)  recipe_planner/utils.py:157 */
#define OC_LEVEL0 0      /* E2E_BRTDP planner levels, oc_subtask.level */
#define OC_LEVEL1 1

/* One planner configuration (set_settings(env, subtask, subtask_agent_names)). */
typedef struct {
    int32_t kind;          /* OC_SUB_* */
    int32_t num_agents;    /* 1 or 2 (is_joint) */
    uint8_t agent[2];      /* subtask agent indices, ascending (sim_agents order) */
    uint8_t start_mask[2]; /* start_obj content mask (Chop, Deliver: [0]); Merge: start_obj[0], [1] */
    uint8_t goal_mask;     /* goal_obj content mask (navigation_planner/utils.py:181-246) */
    uint8_t goal_count;    /* cur_obj_count of _define_goal_state at set_settings */
    uint8_t level;         /* planner level (e2e_brtdp.py:383-406): OC_LEVEL0 (agents outside the
                              subtask become AgentCounters, their items leave) or OC_LEVEL1 (every
                              agent stays; none may be moved into).  oc_rollout only; the other
                              entry points take OC_LEVEL0 */
    uint8_t reserved;
} oc_subtask;

/* rollout flags (per row) */
#define OC_ROLL_LEGAL 0x01  /* the action is in get_actions(state) (joint: both single-legal and
                               is_collision all True) */
#define OC_ROLL_GOAL 0x02   /* is_goal_state(T(state, action)); 0 on OC_ROLL_ASSERT rows */
#define OC_ROLL_ASSERT 0x04 /* joint: the two agents end co-located (the reference's
                               AssertionError at e2e_brtdp.py:143; state_out still written) */
#define OC_ROLL_RAISES 0x08 /* the reference raises configuring the planner: two agents outside the
                               subtask stand on one square (World.remove of the same Floor twice,
                               gym_cooking/utils/world.py:307-315); row copied unchanged, bound 0 */
#define OC_ROLL_BADALLOC 0x80 /* alloc id >= num_subtasks: row copied unchanged, bound 0 */

/* One rollout transition per row e < B:
 *   state_in   : states in the oc_layout (real or already Level-0 states)
 *   state_out  : the Level-0 next state: agents outside the subtask keep their location with
 *                hold = OC_HOLD_NONE and their held items dead; t and flags copied
 *   actions    : u8 [A][pitch] codes; only the subtask agents' rows are read
 *   alloc      : nullable u8 [pitch] index into subtasks per row (NULL: subtasks[0])
 *   subtasks   : host array of num_subtasks (<= OC_MAX_SUBTASKS) planner configurations
 *   out_flags  : u8 [pitch] OC_ROLL_* ;  lower_bound : f32 [pitch], the lower bound of the
 *                next state before the planner's cost factor (value_init: v_l = 1.1*lb - 1.09,
 *                v_u = 6.05*lb; goal states have value 0) */
/* Level: with OC_LEVEL1 in a configuration's `level` the row keeps every agent (the planner's
 * Level-1 env, e2e_brtdp.py:383-392): nothing is removed, no agent's cell may be moved into. */
int oc_rollout(const oc_handle* h, const void* state_in, void* state_out, const uint8_t* actions,
               const uint8_t* alloc, const oc_subtask* subtasks, int32_t num_subtasks,
               uint8_t* out_flags, float* lower_bound, int64_t B, void* stream);

/* ---------------------------------------------------------------------------------------
 * Bayesian-delegation action likelihood: per row,
 *   BayesianDelegator.prob_nav_actions(obs_tm1, actions_tm1, subtask, subtask_agent_names,
 *                                      beta, no_level_1=True)
 *     gym_cooking/delegation_planner/bayesian_delegator.py:461-689
 * for a planner whose values are all value_init's (a fresh E2E_BRTDP, e2e_brtdp.py:678-729):
 *   Q(s, a) = cost(a) + v_l(T(s, a)),  cost = 1.0 + 0.1 per moving subtask agent (:816-826),
 *   v_l = 0 on goal states, else 1.1 * lower_bound - 1.09;
 *   p = softmax(beta * (Q(s, taken) - Q(s, a')))[taken] over get_actions(s) (joint actions of a
 *   pair that contains self_agent keep the other agent's taken action, :676-680);
 *   subtask None (one agent): softmax(beta * [p0, (1 - p0) / n, ...])[taken != (0,0)], n = the
 *   self agent's movable actions in the full (not Level-0) state.
 * The reference's own bayes_update runs Level 1 (other agents' planners predict their moves)
 * and BRTDP updates its values between calls; neither is restated here.
 * ------------------------------------------------------------------------------------- */
#define OC_LIK_OK 0x01       /* likelihood computed */
#define OC_LIK_RAISES 0x04   /* the reference raises: taken action not in get_actions, a joint T
                                co-location assert, two removed agents on one square (Level-0
                                configuration), or None for two agents */
#define OC_LIK_ZERODIV 0x08  /* None subtask and the self agent has no movable action */
#define OC_LIK_BADALLOC 0x80 /* alloc id >= num_subtasks */

/*   state        : obs_tm1 states (oc_layout), B rows
 *   taken        : u8 [A][pitch] executed actions actions_tm1 (env.agent_actions, :770)
 *   alloc/subtasks/num_subtasks : as oc_rollout (goal_count = the planner's cur_obj_count)
 *   self_agent   : the delegating agent's index (BayesianDelegator.agent_name)
 *   likelihood   : f64 [pitch]; out_flags : u8 [pitch] OC_LIK_* */
int oc_nav_likelihood(const oc_handle* h, const void* state, const uint8_t* taken, const uint8_t* alloc,
                      const oc_subtask* subtasks, int32_t num_subtasks, int32_t self_agent, double beta,
                      double none_action_prob, double* likelihood, uint8_t* out_flags, int64_t B, void* stream);

/* Which kernel oc_nav_likelihood runs on handle h: OC_LIK_FORM_AUTO (the default: the
 * compacted form, whose rollouts are spread over the wave, where the level's tables leave it
 * the LDS; else the grouped form) or OC_LIK_FORM_GROUPED (the grouped form always).  The two
 * give the same bits; this exists so a test can run the grouped form on any level. */
#define OC_LIK_FORM_AUTO 0
#define OC_LIK_FORM_GROUPED 1
int oc_set_likelihood_form(oc_handle* h, int32_t form);

/* The level's static reachability graph, World.make_reachability_graph (utils/world.py:67-108),
 * as built by oc_create: nodes are (cell, approach) with approach 0..3 = World.NAV_ACTIONS (the
 * side a collidable square is reached from) and 4 = (0, 0) (a Floor square).  Host data; works
 * without a device.
 *   num_nodes : out, n
 *   node_of   : nullable u16 [W*H*5]: node id of (cell, approach), 0xFFFF = not a node
 *   dist      : nullable u8 [n][n]: nx.shortest_path_length between nodes, 0xFF = no path
 * World.get_lower_bound_between(_helper) (world.py:115-283) evaluates over exactly this table.
 * The planner kernels keep the distance table in LDS for a graph of at most 360 nodes, in device
 * memory past that (a narrow level: every node its 255 cells can make; a wide one: up to 5,120).
 * A graph with a BFS distance of 255 or more (a maze kitchen's corridors) has u16 tables, in
 * device memory (ABI 10; ABI 9 refused it): oc_reachability then fails with OC_ELEVEL when
 * `dist` is given (the u8 table cannot hold it), and oc_reachability16 gives it. */
int oc_reachability(const oc_handle* h, int32_t* num_nodes, uint16_t* node_of, int64_t node_of_len, uint8_t* dist,
                    int64_t dist_len);
/* The same with u16 distances (0xFFFF = no path), for every level (ABI 10). */
int oc_reachability16(const oc_handle* h, int32_t* num_nodes, uint16_t* node_of, int64_t node_of_len, uint16_t* dist,
                      int64_t dist_len);

/* ---------------------------------------------------------------------------------------
 * Subtask bounds on full environment states (no planner Level-0 view): for every env e and
 * every configuration i of the call,
 *   lower_bound[i][e] = env.get_lower_bound_for_subtask_given_objs(subtask, agents, start_obj,
 *                        goal_obj, subtask_action_obj)
 *                       gym_cooking/envs/overcooked_environment.py:594-664, with
 *                       get_AB_locs_given_objs :480-589 and World.get_lower_bound_between(_helper)
 *                       utils/world.py:115-283 (None: perimeter + 1 + holding penalty)
 *   doable[i][e]      = BayesianDelegator.subtask_alloc_is_doable(env, subtask, agents)
 *                       delegation_planner/bayesian_delegator.py:98-156 (None: 1; else the
 *                       get_lower_bound_between distance < world.perimeter), the feasibility
 *                       test of prune_subtask_allocs (:200-260)
 * Replaces the per-(state, allocation) Python calls of the delegation planner's prior setup
 * (set_priors -> prune_subtask_allocs) and of a drop-in env's planner queries.
 *   state       : B states (oc_layout)
 *   subtasks    : host array of num_subtasks (<= OC_MAX_SUBTASKS); goal_count is ignored
 *   lower_bound : f32 [num_subtasks][pitch];  doable : u8 [num_subtasks][pitch]
 * ------------------------------------------------------------------------------------- */
int oc_subtask_bounds(const oc_handle* h, const void* state, const oc_subtask* subtasks, int32_t num_subtasks,
                      float* lower_bound, uint8_t* doable, int64_t B, void* stream);

/* ---------------------------------------------------------------------------------------
 * Image observation: what GameImage.get_image_obs returns after on_render
 *   gym_cooking/misc/game/gameimage.py:31-51, game.py:56-186
 * per env: the static level image (floor fill, counters with a 1-px border, delivery and
 * cutboard sprites; built once on the host by gym_cooking_amd/render.py), then every item
 * that is not held (tile-size sprite; a plate first, its contents at the container size /
 * offset), then each agent in order with its held item (holding size / offset), each sprite
 * blended per pixel with SDL 1.2's ALPHA_BLEND (d += ((s - d) * a + 255) >> 8, a = 0 skipped).
 * Output u8 [B][H*tile][W*tile][3]; byte c of a pixel = source channel (chan_map >> 8c) & 0xFF
 * (0 R, 1 G, 2 B, 3 constant 0).  The reference reads its 0x00RRGGBB pixels through
 * pygame.Color(int) (0xRRGGBBAA) and stores (g, b, r) = (R, G, 0): OC_CHAN_REFERENCE.
 * ------------------------------------------------------------------------------------- */
#define OC_RENDER_SIZES 4          /* tile, container, holding, holding container */
#define OC_CHAN_RGB 0x00020100u
#define OC_CHAN_REFERENCE 0x00030100u

typedef struct {
    int32_t tile;                         /* pixels per cell (Game.scale, 80; a multiple of 16) */
    int32_t size[OC_RENDER_SIZES];        /* sprite edge per size class: 80, 56, 40, 28 */
    int32_t offset[OC_RENDER_SIZES];      /* sprite origin inside its cell: 0, 12, 40, 46 */
    int32_t food_base[OC_RENDER_SIZES];   /* atlas pixel offset of food sprite 0 of each size class;
                                             food sprite i of class c at food_base[c] + i*size[c]^2 */
    int32_t plate_off[2];                 /* plate sprite at tile size, at holding size */
    int32_t agent_off[OC_MAX_AGENTS];     /* agent-<colour> sprite (utils/agent.py:25 colour order) */
    uint8_t food_sprite[128];             /* plate-less content mask -> food sprite index, 0xFF none */
    uint32_t chan_map;                    /* OC_CHAN_* */
} oc_render_desc;

/*   state      : B states (oc_layout)
 *   atlas      : device u32 RGBA sprites (R | G<<8 | B<<16 | A<<24), laid out as desc says
 *   background : device u32 RGBX [H*tile][W*tile], the static level image
 *   out        : device u8 [B][H*tile][W*tile][3] */
int oc_render(const oc_handle* h, const void* state, const uint32_t* atlas, const uint32_t* background,
              const oc_render_desc* desc, uint8_t* out, int64_t B, void* stream);

/* oc_render with the draw order of objects that share a square (Game.on_render draws the
 * objects not held in world.objects order, game.py:62-74: name groups in first-insertion
 * order, each in insertion order -- episode history, world.py:304-315, interact.py:46-52).
 *   draw_rank : device u8 [K][pitch] or NULL; objects of one square are drawn in ascending
 *               rank, ties in slot order.  NULL: slot order (oc_render).  The host side's
 *               render.DrawOrder replays the reference's order from consecutive states. */
int oc_render_ordered(const oc_handle* h, const void* state, const uint8_t* draw_rank, const uint32_t* atlas,
                      const uint32_t* background, const oc_render_desc* desc, uint8_t* out, int64_t B,
                      void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OC_ENGINE_H_ */
