/*
 * oracle/oc_oracle.c -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * A scalar CPU restatement of the reference environment step of deletfsi/gym-cooking
 * (pure Python; nothing to compile), written object-by-object after the reference so that
 * each routine can be read against the line it restates.  It is the parity checker for the
 * HIP engine (tests/) and the CPU baseline leg of bench.py.  Only tests/, smoke() and
 * bench.py's cpu_baseline may load it; the product path (liboc_engine.so) never does.
 *
 * Pinning: tests/test_oracle_golden.py replays every fixture under tests/golden/ (generated
 * by importing the reference itself, tests/golden/gen_golden.py) and requires bit-exact
 * agreement of the canonical state, executed actions, collision masks and flags.
 *
 * State layout = include/oc_engine.h oc_layout (byte planes, canonical App. A.11 fields).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>

#include "../include/oc_engine.h"

#define NFOOD 3 /* Tomato, Lettuce, Onion */

typedef struct { int x, y; } Loc;

/* core.Object (gym_cooking/utils/core.py:130-219).  Contents: a count of each food type
 * with the FRESH_CHOPPED state index of those foods (core.py:250-252, 310-346; the foods of
 * one object share a state: a merge takes only foods in their last state, core.py:222-241),
 * plus a plate count.  Under OC_ENC_PRESENCE a level holds at most one of each food. */
typedef struct {
    int alive; /* present in World.objects */
    Loc location;
    int is_held;
    int food_count[NFOOD];
    int food_state[NFOOD]; /* 0 = Fresh, 1 = Chopped */
    int plates;
} Obj;

/* utils.agent.SimAgent (gym_cooking/utils/agent.py:371-423) */
typedef struct {
    Loc location;
    int holding; /* index into objs, -1 = None */
    Loc action;
} Agent;

typedef struct {
    const oc_level_desc* L;
    int A, K;
    int t;
    Obj objs[OC_MAX_ITEMS];
    Agent agents[OC_MAX_AGENTS];
    /* planner Level-0 view (e2e_brtdp.py:389-406): agents outside the subtask are removed
     * from sim_agents and their Floor becomes an AgentCounter; 0 / all-active on the env step */
    int ac_cell[OC_MAX_AGENTS]; /* AgentCounter cells (-1 none), one per removed agent */
    int active[OC_MAX_AGENTS];
} Env;

static const Loc NAV[5] = {{0, 1}, {0, -1}, {-1, 0}, {1, 0}, {0, 0}};

static int loc_eq(Loc a, Loc b) { return a.x == b.x && a.y == b.y; }
static Loc loc_add(Loc a, Loc b) { Loc r = {a.x + b.x, a.y + b.y}; return r; }

static int action_code(Loc a) {
    for (int i = 0; i < 5; ++i)
        if (loc_eq(a, NAV[i])) return i;
    abort();
}

/* World.get_gridsquare_at (world.py:421-430): the unique GridSquare at location. The
 * reference asserts when there is none (off-grid); step_one catches that case first. */
static int gridsquare_at(const Env* e, Loc l) {
    if (l.x < 0 || l.y < 0 || l.x >= e->L->width || l.y >= e->L->height) abort();
    const int c = l.y * e->L->width + l.x;
    for (int a = 0; a < OC_MAX_AGENTS; ++a)
        if (e->ac_cell[a] == c) return OC_TILE_COUNTER; /* AgentCounter (core.py:79-93) */
    return e->L->tiles[c];
}

/* GridSquare.collidable: only Floor is walkable (core.py:34, 64) */
static int collidable(int tile) { return tile != OC_TILE_FLOOR; }

/* World.inbounds (world.py:432-436) */
static Loc inbounds(const Env* e, Loc l) {
    Loc r;
    r.x = l.x < 0 ? 0 : (l.x > e->L->width - 1 ? e->L->width - 1 : l.x);
    r.y = l.y < 0 ? 0 : (l.y > e->L->height - 1 ? e->L->height - 1 : l.y);
    return r;
}

/* World.is_occupied (world.py:285-290): an un-held Object at location */
static int is_occupied(const Env* e, Loc l) {
    for (int i = 0; i < e->K; ++i)
        if (e->objs[i].alive && loc_eq(e->objs[i].location, l) && !e->objs[i].is_held) return 1;
    return 0;
}

/* World.get_object_at(location, None, find_held_objects) (world.py:389-419); returns -1
 * where the reference's `assert len(objs) == 1` would fail. */
static int object_at(const Env* e, Loc l, int find_held) {
    int found = -1, n = 0;
    for (int i = 0; i < e->K; ++i)
        if (e->objs[i].alive && loc_eq(e->objs[i].location, l) && e->objs[i].is_held == find_held) {
            found = i;
            ++n;
        }
    return n == 1 ? found : -1;
}

static int n_contents(const Obj* o) {
    int n = o->plates;
    for (int f = 0; f < NFOOD; ++f) n += o->food_count[f];
    return n;
}

/* The content mask of an object in the level's encoding (include/oc_engine.h OC_ENC_*): the
 * canonical identity of Object.full_name (core.py:143-171). */
static int obj_mask_enc(const Obj* o, int enc) {
    if (enc == OC_ENC_COUNTS) {
        static const int unit[NFOOD] = {OC_MC_TOMATO, OC_MC_LETTUCE, OC_MC_ONION};
        int m = o->plates ? OC_MC_PLATE : 0, fresh = 0;
        for (int f = 0; f < NFOOD; ++f) {
            m += o->food_count[f] * unit[f];
            if (o->food_count[f] && o->food_state[f] == 0) fresh = 1;
        }
        return m | (fresh ? OC_MC_FRESH : 0);
    }
    int m = o->plates ? OC_M_PLATE : 0;
    for (int f = 0; f < NFOOD; ++f)
        if (o->food_count[f]) m |= (1 << f) | (o->food_state[f] << (f + OC_M_CHOPPED_SHIFT));
    return m;
}

static void obj_set_mask(Obj* o, int m, int enc) {
    if (enc == OC_ENC_COUNTS) {
        o->plates = (m & OC_MC_PLATE) ? 1 : 0;
        for (int f = 0; f < NFOOD; ++f) {
            o->food_count[f] = (m >> (2 * f)) & 3;
            o->food_state[f] = (m & OC_MC_FRESH) ? 0 : 1;
        }
        return;
    }
    o->plates = (m & OC_M_PLATE) ? 1 : 0;
    for (int f = 0; f < NFOOD; ++f) {
        o->food_count[f] = (m >> f) & 1;
        o->food_state[f] = (m >> (f + OC_M_CHOPPED_SHIFT)) & 1;
    }
}

/* Food.done (core.py:293-296): state index is the last of FRESH_CHOPPED */
static int food_done(const Obj* o, int f) { return o->food_state[f] == 1; }

/* Object.needs_chopped (core.py:176-178) -> Food.needs_chopped (core.py:285-291) /
 * Plate.needs_chopped (core.py:365-366) */
static int needs_chopped(const Obj* o) {
    if (n_contents(o) > 1) return 0;
    if (o->plates) return 0;
    for (int f = 0; f < NFOOD; ++f)
        if (o->food_count[f]) return o->food_state[f] == 0; /* next state is Chopped */
    return 0;
}

/* Object.chop (core.py:187-192) */
static void chop(Obj* o) {
    for (int f = 0; f < NFOOD; ++f)
        if (o->food_count[f]) o->food_state[f] += 1;
}

/* Object.is_deliverable (core.py:214-219) */
static int is_deliverable(const Obj* o) {
    for (int f = 0; f < NFOOD; ++f)
        if (o->food_count[f] && !food_done(o, f)) return 0;
    return n_contents(o) > 1; /* is_merged */
}

/* mergeable (core.py:222-241): drop up to one Plate; a second Plate => False; otherwise
 * every remaining content must be in its last state. */
static int mergeable(const Obj* a, const Obj* b) {
    int plates = a->plates + b->plates;
    if (plates >= 2) return 0;
    for (int f = 0; f < NFOOD; ++f) {
        if (a->food_count[f] && !food_done(a, f)) return 0;
        if (b->food_count[f] && !food_done(b, f)) return 0;
    }
    return 1;
}

/* Object.merge (core.py:194-202): contents += other's contents (merged foods are all in their
 * last state, so the counts add up under one state) */
static void merge(Obj* a, const Obj* b) {
    a->plates += b->plates;
    for (int f = 0; f < NFOOD; ++f)
        if (b->food_count[f]) {
            a->food_count[f] += b->food_count[f];
            a->food_state[f] = b->food_state[f];
        }
}

/* SimAgent.acquire (agent.py:408-414) */
static void agent_acquire(Env* e, Agent* ag, int obj) {
    if (ag->holding < 0) {
        ag->holding = obj;
        e->objs[obj].is_held = 1;
        e->objs[obj].location = ag->location;
    } else {
        merge(&e->objs[ag->holding], &e->objs[obj]);
    }
}

/* SimAgent.release (agent.py:416-418) */
static void agent_release(Env* e, Agent* ag) {
    e->objs[ag->holding].is_held = 0;
    ag->holding = -1;
}

/* SimAgent.move_to (agent.py:420-423) */
static void agent_move_to(Env* e, Agent* ag, Loc l) {
    ag->location = l;
    if (ag->holding >= 0) e->objs[ag->holding].location = l;
}

/* interact(agent, world) (utils/interact.py:4-89), world.arglist.play == False */
static void interact(Env* e, Agent* ag) {
    if (loc_eq(ag->action, NAV[OC_ACT_NOOP])) return;                /* :19-20 */
    Loc target = inbounds(e, loc_add(ag->location, ag->action));     /* :22 */
    int gs = gridsquare_at(e, target);                               /* :24 */
    if (gs == OC_TILE_FLOOR) {                                       /* :28-30 */
        agent_move_to(e, ag, target);
    } else if (ag->holding >= 0) {                                   /* :33 */
        if (gs == OC_TILE_DELIVERY) {                                /* :35-40 */
            Obj* obj = &e->objs[ag->holding];
            if (is_deliverable(obj)) {
                obj->location = target; /* Delivery.acquire (core.py:110-112) */
                agent_release(e, ag);
            }
        } else if (is_occupied(e, target)) {                         /* :43-56 */
            int o = object_at(e, target, 0);
            if (o < 0) abort();
            if (mergeable(&e->objs[ag->holding], &e->objs[o])) {
                e->objs[o].alive = 0;   /* world.remove(obj); gs.release() */
                /* world.remove(agent.holding) + world.insert(agent.holding): the holder's
                 * object survives under its new name (identity kept in its slot). */
                agent_acquire(e, ag, o); /* holding.merge(obj) */
            }
        } else {                                                     /* :60-70 */
            Obj* obj = &e->objs[ag->holding];
            if (gs == OC_TILE_CUTBOARD && needs_chopped(obj)) {
                chop(obj);
            } else {
                obj->location = target; /* gs.acquire(obj) (core.py:50-52) */
                agent_release(e, ag);
            }
        }
    } else {                                                         /* :73-89 */
        if (is_occupied(e, target) && gs != OC_TILE_DELIVERY) {
            int o = object_at(e, target, 0);
            if (o < 0) abort();
            agent_acquire(e, ag, o); /* gs.release(); agent.acquire(obj) */
        }
    }
}

/* OvercookedEnvironment.is_collision (overcooked_environment.py:671-718) */
static void is_collision(const Env* e, Loc l1, Loc l2, Loc a1, Loc a2, int exec_[2]) {
    exec_[0] = 1;
    exec_[1] = 1;
    Loc n1 = loc_add(l1, a1);
    if (collidable(gridsquare_at(e, n1))) n1 = l1;
    Loc n2 = loc_add(l2, a2);
    if (collidable(gridsquare_at(e, n2))) n2 = l2;
    Loc zero = NAV[OC_ACT_NOOP];
    if (loc_eq(n1, n2)) {
        if (loc_eq(n1, l1) && !loc_eq(a1, zero)) {
            exec_[1] = 0;
        } else if (loc_eq(n2, l2) && !loc_eq(a2, zero)) {
            exec_[0] = 0;
        } else {
            exec_[0] = 0;
            exec_[1] = 0;
        }
    } else if (loc_eq(l1, n2) && loc_eq(l2, n1)) {
        exec_[0] = 0;
        exec_[1] = 0;
    }
}

/* OvercookedEnvironment.check_collisions (overcooked_environment.py:724-762); returns the
 * pair mask in itertools.combinations order. */
static int check_collisions(Env* e) {
    int execute[OC_MAX_AGENTS];
    for (int i = 0; i < e->A; ++i) execute[i] = 1;
    int pair = 0, mask = 0;
    for (int i = 0; i < e->A; ++i)
        for (int j = i + 1; j < e->A; ++j, ++pair) {
            int ex[2];
            is_collision(e, e->agents[i].location, e->agents[j].location, e->agents[i].action,
                         e->agents[j].action, ex);
            if (!ex[0]) execute[i] = 0;
            if (!ex[1]) execute[j] = 0;
            if (!(ex[0] && ex[1])) mask |= 1 << pair; /* CollisionRepr appended */
        }
    for (int i = 0; i < e->A; ++i)
        if (!execute[i]) e->agents[i].action = NAV[OC_ACT_NOOP];
    return mask;
}

/* new_obs = copy.copy(self) (overcooked_environment.py:289 -> __copy__ :108-113): every
 * holding agent must find exactly one held object at its location (world.py:417). */
static int copy_would_raise(const Env* e) {
    for (int i = 0; i < e->A; ++i)
        if (e->agents[i].holding >= 0 && object_at(e, e->agents[i].location, 1) < 0) return 1;
    return 0;
}

/* done() (overcooked_environment.py:316-363) + reward() (:365-376). Returns flags. */
static int done_flags(const Env* e, int max_T) {
    if (e->t >= max_T && max_T) return OC_FLAG_DONE; /* :328-332 */
    const oc_level_desc* L = e->L;
    int dcell = -1; /* first Delivery in World.objects order = map scan order (:349) */
    for (int c = 0; c < L->width * L->height; ++c)
        if (L->tiles[c] == OC_TILE_DELIVERY) { dcell = c; break; }
    Loc dloc = {dcell % L->width, dcell / L->width};
    for (int g = 0; g < L->num_goals; ++g) { /* every Deliver subtask (:344-359) */
        int gm = L->goal_mask[g], ok = 0;
        for (int i = 0; i < e->K; ++i) {
            const Obj* o = &e->objs[i];
            if (!o->alive || !loc_eq(o->location, dloc)) continue;
            if (obj_mask_enc(o, L->encoding) == gm) ok = 1; /* goal_obj == o (core.py:143-148) */
        }
        if (!ok) return 0;
    }
    return OC_FLAG_DONE | OC_FLAG_SUCCESS;
}

/* ---- canonical layout <-> object model ---- */

typedef struct {
    const oc_level_desc* L;
    int A, K, max_T;
    int64_t pitch;
} Cfg;

static void unpack(const Cfg* c, const uint8_t* s, int64_t e, Env* env, int* flags) {
    const int64_t P = c->pitch;
    env->L = c->L;
    env->A = c->A;
    env->K = c->K;
    const int A = c->A, K = c->K;
    const uint8_t* ax = s + 0 * A * P;
    const uint8_t* ay = s + 1 * A * P;
    const uint8_t* ah = s + 2 * A * P;
    /* a wide level (more than OC_MAX_NARROW_CELLS cells): u16 cells, high bytes in K planes
     * after the low ones (oc_layout.plane_item_loc_hi) */
    const int wide = c->L->width * c->L->height > OC_MAX_NARROW_CELLS, LK = wide ? 2 * K : K;
    const uint8_t* il = s + 3 * A * P;
    const uint8_t* ilh = s + (3 * A + K) * P;
    const uint8_t* im = s + (3 * A + LK) * P;
    const uint16_t* tp = (const uint16_t*)(s + (3 * A + LK + K) * P);
    const uint8_t* fl = s + (3 * A + LK + K + 2) * P;
    env->t = tp[e];
    *flags = fl[e];
    for (int k = 0; k < K; ++k) {
        Obj* o = &env->objs[k];
        memset(o, 0, sizeof(*o));
        const int loc = il[k * P + e] | (wide ? ilh[k * P + e] << 8 : 0), m = im[k * P + e];
        o->alive = loc != (wide ? (int)OC_LOC_DEAD16 : (int)OC_LOC_DEAD);
        o->location.x = loc % c->L->width;
        o->location.y = loc / c->L->width;
        obj_set_mask(o, m, c->L->encoding);
    }
    for (int a = 0; a < A; ++a) {
        Agent* g = &env->agents[a];
        g->location.x = ax[a * P + e];
        g->location.y = ay[a * P + e];
        uint8_t h = ah[a * P + e];
        g->holding = h == OC_HOLD_NONE ? -1 : h;
        if (g->holding >= K) abort();
        g->action = NAV[OC_ACT_NOOP];
    }
    for (int a = 0; a < A; ++a)
        if (env->agents[a].holding >= 0) env->objs[env->agents[a].holding].is_held = 1;
    for (int a = 0; a < OC_MAX_AGENTS; ++a) {
        env->ac_cell[a] = -1;
        env->active[a] = 1;
    }
}

static void pack(const Cfg* c, const Env* env, int flags, uint8_t* s, int64_t e) {
    const int64_t P = c->pitch;
    const int A = c->A, K = c->K;
    uint8_t* ax = s + 0 * A * P;
    uint8_t* ay = s + 1 * A * P;
    uint8_t* ah = s + 2 * A * P;
    const int wide = c->L->width * c->L->height > OC_MAX_NARROW_CELLS, LK = wide ? 2 * K : K;
    uint8_t* il = s + 3 * A * P;
    uint8_t* ilh = s + (3 * A + K) * P;
    uint8_t* im = s + (3 * A + LK) * P;
    uint16_t* tp = (uint16_t*)(s + (3 * A + LK + K) * P);
    uint8_t* fl = s + (3 * A + LK + K + 2) * P;
    tp[e] = (uint16_t)env->t;
    fl[e] = (uint8_t)flags;
    for (int a = 0; a < A; ++a) {
        ax[a * P + e] = (uint8_t)env->agents[a].location.x;
        ay[a * P + e] = (uint8_t)env->agents[a].location.y;
        ah[a * P + e] = env->agents[a].holding < 0 ? OC_HOLD_NONE : (uint8_t)env->agents[a].holding;
    }
    for (int k = 0; k < K; ++k) {
        const Obj* o = &env->objs[k];
        if (!o->alive) {
            il[k * P + e] = OC_LOC_DEAD;
            if (wide) ilh[k * P + e] = OC_LOC_DEAD;
            im[k * P + e] = 0;
            continue;
        }
        const int cell = o->location.y * c->L->width + o->location.x;
        il[k * P + e] = (uint8_t)cell;
        if (wide) ilh[k * P + e] = (uint8_t)(cell >> 8);
        im[k * P + e] = (uint8_t)obj_mask_enc(o, c->L->encoding);
    }
}

/* reset() (overcooked_environment.py:201-250) -> load_level (:130-198) template */
static void template_env(const Cfg* c, Env* env) {
    memset(env, 0, sizeof(*env));
    env->L = c->L;
    env->A = c->A;
    env->K = c->K;
    env->t = 0;
    for (int k = 0; k < c->K; ++k) {
        Obj* o = &env->objs[k];
        if (k >= c->L->num_items) { o->alive = 0; continue; }
        o->alive = 1;
        o->location.x = c->L->item_cell[k] % c->L->width;
        o->location.y = c->L->item_cell[k] / c->L->width;
        obj_set_mask(o, c->L->item_mask[k], c->L->encoding);
    }
    for (int a = 0; a < c->A; ++a) {
        env->agents[a].location.x = c->L->spawn_x[a];
        env->agents[a].location.y = c->L->spawn_y[a];
        env->agents[a].holding = -1;
        env->agents[a].action = NAV[OC_ACT_NOOP];
    }
    for (int a = 0; a < OC_MAX_AGENTS; ++a) env->active[a] = 1;
}

/* step() (overcooked_environment.py:255-306) for env e. */
static void step_one(const Cfg* c, const uint8_t* sin, uint8_t* sout, const uint8_t* act,
                     uint8_t* exec_out, uint8_t* coll_out, int64_t e) {
    Env env;
    int flags;
    unpack(c, sin, e, &env, &flags);
    const int64_t P = c->pitch;
    if (flags & OC_FLAG_DONE) { /* next-step auto-reset (build definition) */
        template_env(c, &env);
        pack(c, &env, 0, sout, e);
        for (int a = 0; a < c->A; ++a)
            if (exec_out) exec_out[a * P + e] = OC_ACT_NOOP;
        if (coll_out) coll_out[e] = 0;
        return;
    }
    env.t += 1; /* :257 */
    for (int a = 0; a < c->A; ++a) { /* :263-264 */
        int code = act[a * P + e];
        env.agents[a].action = NAV[code > OC_ACT_NOOP ? OC_ACT_NOOP : code];
    }
    if (c->A >= 2) { /* check_collisions -> is_collision looks up the unclamped next square */
        int off = 0;
        for (int a = 0; a < c->A; ++a) {
            Loc n = loc_add(env.agents[a].location, env.agents[a].action);
            off |= n.x < 0 || n.y < 0 || n.x >= c->L->width || n.y >= c->L->height;
        }
        if (off) { /* get_gridsquare_at asserts (world.py:429): step raises before anything moves */
            pack(c, &env, OC_FLAG_DONE | OC_FLAG_ERR, sout, e); /* t advanced (:257), nothing else */
            for (int a = 0; a < c->A; ++a)
                if (exec_out) exec_out[a * P + e] = OC_ACT_NOOP;
            if (coll_out) coll_out[e] = 0;
            return;
        }
    }
    int cmask = check_collisions(&env); /* :267 */
    int ex[OC_MAX_AGENTS];
    for (int a = 0; a < c->A; ++a) { /* execute_navigation :767-770 */
        interact(&env, &env.agents[a]);
        ex[a] = action_code(env.agents[a].action);
    }
    int out_flags;
    if (copy_would_raise(&env))
        out_flags = OC_FLAG_DONE | OC_FLAG_ERR;
    else
        out_flags = done_flags(&env, c->max_T); /* :295-298 */
    pack(c, &env, out_flags, sout, e);
    for (int a = 0; a < c->A; ++a)
        if (exec_out) exec_out[a * P + e] = (uint8_t)ex[a];
    if (coll_out) coll_out[e] = (uint8_t)cmask;
}

typedef struct {
    const Cfg* c;
    const uint8_t* sin;
    uint8_t* sout;
    const uint8_t* act;
    uint8_t* ex;
    uint8_t* coll;
    int64_t lo, hi;
} Job;

static void* run_job(void* p) {
    Job* j = (Job*)p;
    for (int64_t e = j->lo; e < j->hi; ++e) step_one(j->c, j->sin, j->sout, j->act, j->ex, j->coll, e);
    return NULL;
}

/* Batched oracle step over the canonical layout (same semantics as oc_step). */
int oco_step(const oc_level_desc* L, int A, int K, int max_T, const uint8_t* sin, uint8_t* sout,
             const uint8_t* act, uint8_t* exec_out, uint8_t* coll_out, int64_t B, int64_t pitch,
             int nthreads) {
    if (A < 1 || A > OC_MAX_AGENTS || K < 1 || K > OC_MAX_ITEMS || B < 0 || pitch < B) return OC_EINVAL;
    Cfg c = {L, A, K, max_T, pitch};
    if (nthreads < 1) nthreads = 1;
    if (nthreads == 1 || B < 4096) {
        Job j = {&c, sin, sout, act, exec_out, coll_out, 0, B};
        run_job(&j);
        return OC_OK;
    }
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    Job jobs[256];
    int64_t chunk = (B + nthreads - 1) / nthreads;
    for (int i = 0; i < nthreads; ++i) {
        int64_t lo = i * chunk, hi = lo + chunk > B ? B : lo + chunk;
        if (lo > B) lo = B;
        Job j = {&c, sin, sout, act, exec_out, coll_out, lo, hi};
        jobs[i] = j;
        pthread_create(&th[i], NULL, run_job, &jobs[i]);
    }
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    return OC_OK;
}

int oco_reset(const oc_level_desc* L, int A, int K, uint8_t* state, int64_t B, int64_t pitch) {
    if (A < 1 || A > OC_MAX_AGENTS || K < 1 || K > OC_MAX_ITEMS || pitch < B) return OC_EINVAL;
    Cfg c = {L, A, K, 0, pitch};
    Env env;
    template_env(&c, &env);
    for (int64_t e = 0; e < B; ++e) pack(&c, &env, 0, state, e);
    return OC_OK;
}

/* splitmix64 counter RNG (SURVEY 8d synthetic streams) */
static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint8_t oco_action_code(uint64_t seed, uint64_t gid, uint64_t step, uint64_t agent) {
    uint64_t x = seed ^ (gid * 0x9E3779B97F4A7C15ull) ^ (step * 0xC2B2AE3D27D4EB4Full) ^ agent;
    return (uint8_t)(splitmix64(x) % 5u);
}

int oco_gen_actions(int A, uint8_t* act, int64_t B, int64_t pitch, int64_t env_offset, int64_t step,
                    uint64_t seed) {
    for (int a = 0; a < A; ++a)
        for (int64_t e = 0; e < B; ++e)
            act[a * pitch + e] = oco_action_code(seed, (uint64_t)(env_offset + e), (uint64_t)step, (uint64_t)a);
    return OC_OK;
}

/* =========================================================================================
 * Navigation-planner rollout, restated from the reference planner.
 * ========================================================================================= */


static int cell_of(const Env* e, Loc l) { return l.y * e->L->width + l.x; }

/* E2E_BRTDP._configure_planner_level, LEVEL0 branch (e2e_brtdp.py:389-406): every agent
 * not in the subtask leaves sim_agents, the object it holds leaves the world, and its Floor
 * is replaced by an AgentCounter. */
static int level0_view(Env* e, const oc_subtask* s) {
    int raised = 0;
    for (int a = 0; a < e->A; ++a) {
        int in = 0;
        for (int i = 0; i < s->num_agents; ++i) in |= s->agent[i] == a;
        if (in) continue;
        Agent* ag = &e->agents[a];
        e->active[a] = 0;
        if (ag->holding >= 0) {
            e->objs[ag->holding].alive = 0; /* env.world.remove(agent.holding) */
            ag->holding = -1;
        }
        /* env.world.remove(Floor(location)) asserts when a second removed agent stands on an
         * already replaced Floor (world.py:307-315) */
        const int c = cell_of(e, ag->location);
        for (int b = 0; b < OC_MAX_AGENTS; ++b)
            if (e->ac_cell[b] == c) raised = 1;
        e->ac_cell[a] = c; /* Floor -> AgentCounter */
    }
    return raised;
}

/* gs.holding of a non-Floor square: the un-held object on it (Counter / Cutboard /
 * AgentCounter hold at most one; core.py:41-56) or -1 */
static int square_holding(const Env* e, Loc l) {
    for (int i = 0; i < e->K; ++i)
        if (e->objs[i].alive && !e->objs[i].is_held && loc_eq(e->objs[i].location, l)) return i;
    return -1;
}

/* nav_utils.get_single_actions (navigation_planner/utils.py:55-90): is `code` in the list */
static int single_action_legal(const Env* e, int a, int code) {
    if (code == OC_ACT_NOOP) return 1; /* (0, 0) is always appended (:89) */
    const Agent* ag = &e->agents[a];
    Loc nl = inbounds(e, loc_add(ag->location, NAV[code]));
    for (int b = 0; b < e->A; ++b) /* new_loc not in agent_locs (sim_agents of the Level-0 env) */
        if (e->active[b] && loc_eq(e->agents[b].location, nl)) return 0;
    int gs = gridsquare_at(e, nl);
    if (!collidable(gs)) return 1;
    if (gs == OC_TILE_DELIVERY) return 1;
    int o = square_holding(e, nl);
    if (o < 0 && ag->holding >= 0) return 1;
    if (o >= 0 && ag->holding < 0) return 1;
    if (o >= 0 && ag->holding >= 0 && mergeable(&e->objs[ag->holding], &e->objs[o])) return 1;
    return 0;
}

/* E2E_BRTDP.get_actions (e2e_brtdp.py:151-206): is the (joint) action in the list */
static int action_legal(const Env* e, const oc_subtask* s, const int* codes) {
    if (s->kind == OC_SUB_NONE) return codes[0] == OC_ACT_NOOP && (s->num_agents < 2 || codes[1] == OC_ACT_NOOP);
    for (int i = 0; i < s->num_agents; ++i)
        if (!single_action_legal(e, s->agent[i], codes[i])) return 0;
    if (s->num_agents == 2) {
        int ex[2];
        is_collision(e, e->agents[s->agent[0]].location, e->agents[s->agent[1]].location, NAV[codes[0]],
                     NAV[codes[1]], ex);
        if (!(ex[0] && ex[1])) return 0;
    }
    return 1;
}

/* E2E_BRTDP.T (e2e_brtdp.py:103-149): interact for each subtask agent in order, no
 * collision pass; returns 1 where the joint co-location assert (:143) fails. */
static int rollout_T(Env* e, const oc_subtask* s, const int* codes) {
    for (int i = 0; i < s->num_agents; ++i) e->agents[s->agent[i]].action = NAV[codes[i]];
    for (int i = 0; i < s->num_agents; ++i) interact(e, &e->agents[s->agent[i]]);
    if (s->num_agents == 2 && loc_eq(e->agents[s->agent[0]].location, e->agents[s->agent[1]].location)) return 1;
    return 0;
}

/* is_goal_state (e2e_brtdp.py:435-566) */
static int is_goal_state(const Env* e, const oc_subtask* s) {
    if (s->kind == OC_SUB_NONE) return 1;
    int count = 0;
    if (s->kind == OC_SUB_DELIVER) { /* un-held goal objects on a Delivery square */
        for (int i = 0; i < e->K; ++i) {
            const Obj* o = &e->objs[i];
            if (o->alive && !o->is_held && obj_mask_enc(o, e->L->encoding) == s->goal_mask &&
                gridsquare_at(e, o->location) == OC_TILE_DELIVERY)
                ++count;
        }
    } else { /* len(get_all_object_locs(goal_obj)): distinct locations, held or not */
        Loc seen[OC_MAX_ITEMS];
        for (int i = 0; i < e->K; ++i) {
            const Obj* o = &e->objs[i];
            if (!o->alive || obj_mask_enc(o, e->L->encoding) != s->goal_mask) continue;
            int dup = 0;
            for (int j = 0; j < count; ++j) dup |= loc_eq(seen[j], o->location);
            if (!dup) seen[count++] = o->location;
        }
    }
    return count > s->goal_count;
}

/* World.make_reachability_graph (world.py:67-108) over the STATIC level (the graph is built
 * at reset and shared by every copy, world.py:38), as an all-pairs BFS table.  Node id =
 * cell * 5 + d, d = NAV index of the approach direction, 4 = (0, 0) on a Floor. */
#define RG_N (OC_MAX_CELLS * 5)
typedef struct {
    int exists[RG_N];
    int16_t dist[RG_N][RG_N]; /* -1: no path */
} Reach;

static void build_reach(const oc_level_desc* L, Reach* R) {
    const int W = L->width, H = L->height, N = W * H;
    static const int opp[4] = {1, 0, 3, 2};
    int adj[RG_N][8], deg[RG_N];
    memset(R->exists, 0, sizeof(R->exists));
    memset(deg, 0, sizeof(deg));
    for (int c = 0; c < N; ++c) {
        const int x = c % W, y = c / W, coll = L->tiles[c] != OC_TILE_FLOOR;
        if (!coll) R->exists[c * 5 + 4] = 1;
        for (int d = 0; d < 4; ++d) {
            int nx = x + NAV[d].x, ny = y + NAV[d].y;
            nx = nx < 0 ? 0 : (nx > W - 1 ? W - 1 : nx);
            ny = ny < 0 ? 0 : (ny > H - 1 ? H - 1 : ny);
            const int nc = ny * W + nx, ncoll = L->tiles[nc] != OC_TILE_FLOOR;
            if (coll && !ncoll) R->exists[c * 5 + d] = 1;
            (void)opp;
        }
    }
    for (int c = 0; c < N; ++c) { /* edges (undirected; the reference's insertion order does not matter) */
        const int x = c % W, y = c / W, coll = L->tiles[c] != OC_TILE_FLOOR;
        for (int d = 0; d < 4; ++d) {
            int nx = x + NAV[d].x, ny = y + NAV[d].y;
            nx = nx < 0 ? 0 : (nx > W - 1 ? W - 1 : nx);
            ny = ny < 0 ? 0 : (ny > H - 1 ? H - 1 : ny);
            const int nc = ny * W + nx, ncoll = L->tiles[nc] != OC_TILE_FLOOR;
            int u = -1, v = -1;
            if (coll && !ncoll) { u = c * 5 + d; v = nc * 5 + 4; }            /* :96-100 */
            else if (!coll && ncoll) { u = c * 5 + 4; v = nc * 5 + opp[d]; }  /* :101-104 */
            else if (!coll && !ncoll) { u = c * 5 + 4; v = nc * 5 + 4; }      /* :105-107 */
            if (u < 0 || !R->exists[u] || !R->exists[v] || u == v) continue;
            int dup = 0;
            for (int k = 0; k < deg[u]; ++k) dup |= adj[u][k] == v;
            if (!dup) { adj[u][deg[u]++] = v; adj[v][deg[v]++] = u; }
        }
    }
    for (int s0 = 0; s0 < N * 5; ++s0) { /* rows / columns past the level's cells are never read */
        for (int t0 = 0; t0 < N * 5; ++t0) R->dist[s0][t0] = -1;
        if (!R->exists[s0]) continue;
        int q[RG_N], qh = 0, qt = 0;
        R->dist[s0][s0] = 0;
        q[qt++] = s0;
        while (qh < qt) {
            const int u = q[qh++];
            for (int k = 0; k < deg[u]; ++k) {
                const int v = adj[u][k];
                if (R->dist[s0][v] < 0) { R->dist[s0][v] = (int16_t)(R->dist[s0][u] + 1); q[qt++] = v; }
            }
        }
    }
}

/* nx.shortest_path_length; -1 where the reference raises (node missing or no path) */
static int rg_dist(const Reach* R, Loc a, int da, Loc b, int db, int W) {
    const int u = (a.y * W + a.x) * 5 + da, v = (b.y * W + b.x) * 5 + db;
    if (!R->exists[u] || !R->exists[v]) return -1;
    return R->dist[u][v];
}

/* World.get_lower_bound_between_helper (world.py:148-264) + check_bound (:266-283) */
static double lb_helper(const Env* e, const Reach* R, const oc_subtask* s, const Loc* agent_locs, Loc A, Loc B) {
    const int W = e->L->width;
    const double perimeter = 2.0 * (e->L->width + e->L->height);
    double lower = perimeter + 1;
    const int Acoll = collidable(gridsquare_at(e, A)), Bcoll = collidable(gridsquare_at(e, B));
    const int nA = Acoll ? 4 : 1, nB = Bcoll ? 4 : 1;
    for (int ia = 0; ia < nA; ++ia)
        for (int ib = 0; ib < nB; ++ib) {
            const int da = Acoll ? ia : 4, db = Bcoll ? ib : 4;
            double bound;
            if (s->num_agents == 1) {
                const int b1 = rg_dist(R, agent_locs[0], 4, A, da, W);
                const int b2 = rg_dist(R, A, da, B, db, W);
                if (b1 < 0 || b2 < 0) continue; /* except: continue */
                bound = b1 + b2 - 1;
            } else {
                int t;
                const double b1A = (t = rg_dist(R, agent_locs[0], 4, A, da, W)) < 0 ? perimeter : t;
                const double b2A = (t = rg_dist(R, agent_locs[1], 4, A, da, W)) < 0 ? perimeter : t;
                double minA = b1A < b2A ? b1A : b2A;
                const double man = fabs((double)A.x - B.x) + fabs((double)A.y - B.y); /* manhattan_dist -> float */
                const double b1B = (t = rg_dist(R, agent_locs[0], 4, B, db, W)) < 0 ? perimeter : t;
                const double b2B = (t = rg_dist(R, agent_locs[1], 4, B, db, W)) < 0 ? perimeter : t;
                double minB = b1B < b2B ? b1B : b2B;
                if (s->kind == OC_SUB_CHOP || s->kind == OC_SUB_DELIVER) {
                    bound = minA + man - 1;
                } else { /* Merge */
                    if ((b1A == minA && b1B == minB) || (b2A == minA && b2B == minB)) {
                        minA *= 2;
                        minB *= 2;
                    }
                    bound = (minA > minB ? minA : minB) + (man - 1) / 2;
                }
            }
            if (bound < lower) lower = bound;
        }
    return lower > 1 ? lower : 1;
}

/* get_lower_bound_for_subtask_given_objs (overcooked_environment.py:594-664) with
 * get_AB_locs_given_objs (:480-589) and World.get_lower_bound_between (world.py:115-146):
 * returns the get_lower_bound_between distance; *pen_out gets the holding penalty */
static double lower_bound_parts(const Env* e, const Reach* R, const oc_subtask* s, double* pen_out) {
    double penalty = 0.0;
    Loc agent_locs[2];
    int na = 0;
    for (int a = 0; a < e->A; ++a) { /* sim_agents order */
        int in = 0;
        for (int i = 0; i < s->num_agents; ++i) in |= s->agent[i] == a;
        if (!in || !e->active[a]) continue;
        agent_locs[na++] = e->agents[a].location;
        const int h = e->agents[a].holding;
        if (h >= 0 && s->kind != OC_SUB_MERGE) {
            const int m = obj_mask_enc(&e->objs[h], e->L->encoding);
            if (m != s->start_mask[0] && m != s->goal_mask) penalty += 1.0;
        }
    }
    if (penalty > 1) penalty = 1;
    Loc Al[OC_MAX_ITEMS + 2], Bl[OC_MAX_CELLS];
    int nAl = 0, nBl = 0;
    /* get_object_locs(obj, is_held=False) + subtask agents holding obj */
#define OBJ_LOCS(mask, out, n)                                                                    \
    do {                                                                                          \
        for (int i = 0; i < e->K; ++i)                                                            \
            if (e->objs[i].alive && !e->objs[i].is_held && obj_mask_enc(&e->objs[i], e->L->encoding) == (mask))       \
                out[n++] = e->objs[i].location;                                                   \
        for (int a = 0; a < e->A; ++a) {                                                          \
            int in = 0;                                                                           \
            for (int q = 0; q < s->num_agents; ++q) in |= s->agent[q] == a;                       \
            if (in && e->active[a] && e->agents[a].holding >= 0 &&                                \
                obj_mask_enc(&e->objs[e->agents[a].holding], e->L->encoding) == (mask))                               \
                out[n++] = e->agents[a].location;                                                 \
        }                                                                                         \
    } while (0)
    if (s->kind == OC_SUB_CHOP || s->kind == OC_SUB_DELIVER) {
        const int want = s->kind == OC_SUB_CHOP ? OC_TILE_CUTBOARD : OC_TILE_DELIVERY;
        for (int c = 0; c < e->L->width * e->L->height; ++c) /* get_all_object_locs(Cutboard|Delivery) */
            if (e->L->tiles[c] == want) { Bl[nBl].x = c % e->L->width; Bl[nBl].y = c / e->L->width; ++nBl; }
        OBJ_LOCS(s->start_mask[0], Al, nAl);
        if (s->kind == OC_SUB_DELIVER) { /* A_locs not already on a Delivery square */
            int k = 0;
            for (int i = 0; i < nAl; ++i) {
                int in = 0;
                for (int j = 0; j < nBl; ++j) in |= loc_eq(Al[i], Bl[j]);
                if (!in) Al[k++] = Al[i];
            }
            nAl = k;
        }
    } else if (s->kind == OC_SUB_MERGE) {
        OBJ_LOCS(s->start_mask[0], Al, nAl);
        OBJ_LOCS(s->start_mask[1], Bl, nBl);
    }
#undef OBJ_LOCS
    double lower = 2.0 * (e->L->width + e->L->height) + 1;
    for (int i = 0; i < nAl; ++i)
        for (int j = 0; j < nBl; ++j) {
            const double b = lb_helper(e, R, s, agent_locs, Al[i], Bl[j]);
            if (b < lower) lower = b;
        }
    *pen_out = penalty;
    return lower;
}

static double lower_bound(const Env* e, const Reach* R, const oc_subtask* s) {
    double pen;
    const double d = lower_bound_parts(e, R, s, &pen);
    return d + pen;
}

typedef struct {
    Cfg c;
    const Reach* R;
    const uint8_t *sin, *act, *alloc;
    uint8_t *sout, *flags;
    const oc_subtask* subs;
    float* lb;
    int64_t b0, b1;
} RollJob;

static void* run_roll(void* p) {
    RollJob* j = (RollJob*)p;
    const int64_t P = j->c.pitch;
    for (int64_t e = j->b0; e < j->b1; ++e) {
        const oc_subtask* s = &j->subs[j->alloc ? j->alloc[e] : 0];
        Env env;
        int fl;
        unpack(&j->c, j->sin, e, &env, &fl);
        if (s->level == OC_LEVEL0 && level0_view(&env, s)) { /* the reference raises configuring the planner */
            unpack(&j->c, j->sin, e, &env, &fl);
            pack(&j->c, &env, fl, j->sout, e);
            j->flags[e] = OC_ROLL_RAISES;
            j->lb[e] = 0.0f;
            continue;
        }
        int codes[2] = {OC_ACT_NOOP, OC_ACT_NOOP};
        for (int i = 0; i < s->num_agents; ++i) {
            const int c = j->act[s->agent[i] * P + e];
            codes[i] = c > OC_ACT_NOOP ? OC_ACT_NOOP : c;
        }
        if (s->kind == OC_SUB_NONE) codes[0] = codes[1] = OC_ACT_NOOP; /* get_actions -> [(0, 0)] */
        int out = action_legal(&env, s, codes) ? OC_ROLL_LEGAL : 0;
        if (rollout_T(&env, s, codes)) out |= OC_ROLL_ASSERT; /* the reference raised: no goal test */
        else if (is_goal_state(&env, s)) out |= OC_ROLL_GOAL;
        j->lb[e] = (float)lower_bound(&env, j->R, s);
        j->flags[e] = (uint8_t)out;
        pack(&j->c, &env, fl, j->sout, e);
    }
    return NULL;
}

int oco_rollout(const oc_level_desc* L, int A, int K, const uint8_t* sin, uint8_t* sout, const uint8_t* act,
                const uint8_t* alloc, const oc_subtask* subs, int nsub, uint8_t* flags, float* lb, int64_t B,
                int64_t pitch, int nthreads) {
    if (nsub < 1) return -1;
    for (int i = 0; i < nsub; ++i) {
        if (subs[i].num_agents < 1 || subs[i].num_agents > 2) return -1;
        for (int q = 0; q < subs[i].num_agents; ++q)
            if (subs[i].agent[q] >= A) return -1;
        if (subs[i].num_agents == 2 && subs[i].agent[0] >= subs[i].agent[1]) return -1;
    }
    Reach* R = (Reach*)malloc(sizeof(Reach));
    build_reach(L, R);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    RollJob jobs[64];
    for (int t = 0; t < nthreads; ++t) {
        RollJob* j = &jobs[t];
        j->c.L = L; j->c.A = A; j->c.K = K; j->c.max_T = 0; j->c.pitch = pitch;
        j->R = R; j->sin = sin; j->act = act; j->alloc = alloc; j->sout = sout; j->flags = flags;
        j->subs = subs; j->lb = lb;
        j->b0 = B * t / nthreads;
        j->b1 = B * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, run_roll, j);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(R);
    return 0;
}

/* =========================================================================================
 * Bayesian-delegation likelihood (prob_nav_actions, no_level_1, fresh planner values),
 * delegation_planner/bayesian_delegator.py:461-689 over the rollout functions above.
 * ========================================================================================= */

/* E2E_BRTDP.Q(state, action, v_l) (e2e_brtdp.py:736-760) with value_init's v_l; returns 1
 * when T raises (joint co-location) */
static int q_value(const Env* env, const Reach* R, const oc_subtask* s, const int* codes, double* q) {
    Env e2 = *env;
    if (rollout_T(&e2, s, codes)) return 1;
    double cost = 1.0; /* time_cost, + action_cost per non-(0,0) agent action (:816-826) */
    for (int i = 0; i < s->num_agents; ++i)
        if (codes[i] != OC_ACT_NOOP) cost += 0.1;
    double v = 0.0;
    if (!is_goal_state(&e2, s)) {
        const double lower = lower_bound(&e2, R, s) * (1.0 + 0.1);
        v = lower - 1.09;
    }
    *q = cost + 1.0 * v;
    return 0;
}

static int likelihood_row(const Env* env_in, const Reach* R, const oc_subtask* s, const uint8_t* taken_all,
                          int self_agent, double beta, double nap, double* out) {
    Env env = *env_in;
    if (s->kind == OC_SUB_NONE) { /* :629-641 on the full obs_tm1 */
        if (s->num_agents != 1) return OC_LIK_RAISES;
        int n = 0;
        for (int c = 0; c < 4; ++c) n += single_action_legal(&env, self_agent, c);
        if (n == 0) return OC_LIK_ZERODIV;
        const double ap = (1.0 - nap) / n;
        const double x0 = beta * nap, x1 = beta * ap, m = x0 > x1 ? x0 : x1;
        double S = exp(x0 - m);
        for (int k = 0; k < n; ++k) S += exp(x1 - m);
        const int moved = taken_all[s->agent[0]] != OC_ACT_NOOP;
        *out = (moved ? exp(x1 - m) : exp(x0 - m)) / S;
        return OC_LIK_OK;
    }
    if (level0_view(&env, s)) return OC_LIK_RAISES;
    int taken[2] = {OC_ACT_NOOP, OC_ACT_NOOP};
    for (int i = 0; i < s->num_agents; ++i) taken[i] = taken_all[s->agent[i]] > OC_ACT_NOOP ? OC_ACT_NOOP : taken_all[s->agent[i]];
    double old_q;
    if (q_value(&env, R, s, taken, &old_q)) return OC_LIK_RAISES;
    if (!action_legal(&env, s, taken)) return OC_LIK_RAISES; /* assert action in valid_nav_actions */
    int other = -1; /* joint, self in the pair: keep the other agent's action (:676-680) */
    if (s->num_agents == 2) {
        if (s->agent[0] == self_agent) other = 1;
        else if (s->agent[1] == self_agent) other = 0;
    }
    double x[25];
    int nx = 0, ti = -1;
    const int n0 = 5, n1 = s->num_agents == 2 ? 5 : 1;
    for (int a0 = 0; a0 < n0; ++a0)
        for (int a1 = 0; a1 < n1; ++a1) {
            int c[2] = {a0, s->num_agents == 2 ? a1 : OC_ACT_NOOP};
            if (!action_legal(&env, s, c)) continue;
            if (other >= 0 && c[other] != taken[other]) continue;
            double q;
            if (q_value(&env, R, s, c, &q)) return OC_LIK_RAISES;
            if (c[0] == taken[0] && (s->num_agents < 2 || c[1] == taken[1])) ti = nx;
            x[nx++] = beta * (old_q - q);
        }
    if (ti < 0) return OC_LIK_RAISES;
    double m = x[0];
    for (int i = 1; i < nx; ++i) m = x[i] > m ? x[i] : m;
    double S = 0.0;
    for (int i = 0; i < nx; ++i) S += exp(x[i] - m);
    *out = exp(x[ti] - m) / S;
    return OC_LIK_OK;
}

typedef struct {
    Cfg c;
    const Reach* R;
    const uint8_t *sin, *taken, *alloc;
    const oc_subtask* subs;
    int nsub, self_agent;
    double beta, nap;
    double* out;
    uint8_t* flags;
    int64_t b0, b1;
} LikJob;

static void* run_lik(void* p) {
    LikJob* j = (LikJob*)p;
    const int64_t P = j->c.pitch;
    for (int64_t e = j->b0; e < j->b1; ++e) {
        const int ai = j->alloc ? j->alloc[e] : 0;
        j->out[e] = 0.0;
        if (ai >= j->nsub) { j->flags[e] = OC_LIK_BADALLOC; continue; }
        Env env;
        int fl;
        unpack(&j->c, j->sin, e, &env, &fl);
        uint8_t taken[OC_MAX_AGENTS];
        for (int a = 0; a < j->c.A; ++a) taken[a] = j->taken[a * P + e];
        double v = 0.0;
        const int f = likelihood_row(&env, j->R, &j->subs[ai], taken, j->self_agent, j->beta, j->nap, &v);
        j->flags[e] = (uint8_t)f;
        j->out[e] = f == OC_LIK_OK ? v : 0.0;
    }
    return NULL;
}

int oco_nav_likelihood(const oc_level_desc* L, int A, int K, const uint8_t* sin, const uint8_t* taken,
                       const uint8_t* alloc, const oc_subtask* subs, int nsub, int self_agent, double beta, double nap,
                       double* out, uint8_t* flags, int64_t B, int64_t pitch, int nthreads) {
    if (nsub < 1 || self_agent < 0 || self_agent >= A) return -1;
    Reach* R = (Reach*)malloc(sizeof(Reach));
    build_reach(L, R);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    LikJob jobs[64];
    for (int t = 0; t < nthreads; ++t) {
        LikJob* j = &jobs[t];
        j->c.L = L; j->c.A = A; j->c.K = K; j->c.max_T = 0; j->c.pitch = pitch;
        j->R = R; j->sin = sin; j->taken = taken; j->alloc = alloc; j->subs = subs; j->nsub = nsub;
        j->self_agent = self_agent; j->beta = beta; j->nap = nap; j->out = out; j->flags = flags;
        j->b0 = B * t / nthreads;
        j->b1 = B * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, run_lik, j);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(R);
    return 0;
}

/* =========================================================================================
 * Subtask bounds on full states (no Level-0 view): for env e and subtask configuration i,
 *   lb[i*pitch + e]     = get_lower_bound_for_subtask_given_objs (overcooked_environment.py:594-664)
 *   doable[i*pitch + e] = BayesianDelegator.subtask_alloc_is_doable (bayesian_delegator.py:98-156):
 *                         None -> 1, else get_lower_bound_between < world.perimeter
 * ========================================================================================= */
typedef struct {
    Cfg c;
    const Reach* R;
    const uint8_t* sin;
    const oc_subtask* subs;
    int nsub;
    float* lb;
    uint8_t* doable;
    int64_t b0, b1;
} BoundJob;

static void* run_bounds(void* p) {
    BoundJob* j = (BoundJob*)p;
    const int64_t P = j->c.pitch;
    const double perimeter = 2.0 * (j->c.L->width + j->c.L->height);
    for (int64_t e = j->b0; e < j->b1; ++e) {
        Env env;
        int fl;
        unpack(&j->c, j->sin, e, &env, &fl);
        for (int i = 0; i < j->nsub; ++i) {
            const oc_subtask* s = &j->subs[i];
            double pen;
            const double d = lower_bound_parts(&env, j->R, s, &pen);
            j->lb[i * P + e] = (float)(d + pen);
            j->doable[i * P + e] = (uint8_t)(s->kind == OC_SUB_NONE || d < perimeter);
        }
    }
    return NULL;
}

int oco_subtask_bounds(const oc_level_desc* L, int A, int K, const uint8_t* sin, const oc_subtask* subs, int nsub,
                       float* lb, uint8_t* doable, int64_t B, int64_t pitch, int nthreads) {
    if (nsub < 1) return -1;
    for (int i = 0; i < nsub; ++i) {
        if (subs[i].num_agents < 1 || subs[i].num_agents > 2) return -1;
        for (int q = 0; q < subs[i].num_agents; ++q)
            if (subs[i].agent[q] >= A) return -1;
        if (subs[i].num_agents == 2 && subs[i].agent[0] >= subs[i].agent[1]) return -1;
    }
    Reach* R = (Reach*)malloc(sizeof(Reach));
    build_reach(L, R);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    BoundJob jobs[64];
    for (int t = 0; t < nthreads; ++t) {
        BoundJob* j = &jobs[t];
        j->c.L = L; j->c.A = A; j->c.K = K; j->c.max_T = 0; j->c.pitch = pitch;
        j->R = R; j->sin = sin; j->subs = subs; j->nsub = nsub; j->lb = lb; j->doable = doable;
        j->b0 = B * t / nthreads;
        j->b1 = B * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, run_bounds, j);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(R);
    return 0;
}
