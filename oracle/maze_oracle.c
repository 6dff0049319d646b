/*
 * maze_oracle.c -- CPU restatement of the MARL-Maze environment (TEST ONLY).
 *
 * ORACLE / TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product path (marl-maze_amd/) never links,
 * loads or calls it.
 *
 * It restates, in plain C, the algorithm of the reference (rhuangr/MARL-Maze,
 * /root/reference, 2024-10-08) one function at a time; every function cites
 * the reference lines it follows.  It is deliberately a *literal* restatement:
 * the agent's route to the exit is kept as an explicit stack (maze.py:148-154,
 * maze_agent.py:210,232,253-257) rather than the per-cell direction table the
 * HIP kernels use, so agreement between the two checks that shortcut too.
 *
 * Pinned against the golden vectors in tests/golden/ (maze_gen, env_traj,
 * env_ppo), captured by importing the reference (tests/golden/make_golden.py).
 *
 * RNG: CPython's `random` module (Modules/_randommodule.c + Lib/random.py of
 * CPython 3.10, identical in 3.12 for the calls used): MT19937 seeded by
 * init_by_array(abs(seed) as 32-bit words), random() = 53-bit double,
 * getrandbits(k) = genrand>>(32-k), _randbelow(n) by rejection on
 * getrandbits(n.bit_length()), randint(a,b) = a + _randbelow(b-a+1),
 * choice(seq) = seq[_randbelow(len(seq))].
 *
 * Build: see oracle/Makefile (gcc -O2 -fPIC -shared).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MT_N 624
#define MT_M 397
#define OBS_DIM 65
#define MASK_DIM 6
#define ROUTE_CAP 8192
/* maze.py:244-250 / 254-259 loop forever when no cell qualifies (e.g. a tiny
 * maze whose every path cell lies on the shortest path).  Both this oracle and
 * the HIP kernels give up after GEN_TRIES draws with the same protocol: set_end
 * failure -> end = start, path = [start], no key; set_key failure -> no key. */
#define GEN_TRIES 65536

/* ------------------------------------------------------------------------ */
/* CPython MT19937                                                           */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint32_t mt[MT_N];
    int mti;
} PyRng;

static void rng_init_genrand(PyRng* r, uint32_t s) {
    r->mt[0] = s;
    for (int i = 1; i < MT_N; i++)
        r->mt[i] = 1812433253U * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
    r->mti = MT_N;
}

static void rng_init_by_array(PyRng* r, const uint32_t* key, int klen) {
    rng_init_genrand(r, 19650218U);
    int i = 1, j = 0;
    for (int k = (MT_N > klen ? MT_N : klen); k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
        i++;
        j++;
        if (i >= MT_N) { r->mt[0] = r->mt[MT_N - 1]; i = 1; }
        if (j >= klen) j = 0;
    }
    for (int k = MT_N - 1; k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
        i++;
        if (i >= MT_N) { r->mt[0] = r->mt[MT_N - 1]; i = 1; }
    }
    r->mt[0] = 0x80000000U;
}

/* random.seed(int): key = abs(seed) split into little-endian 32-bit words */
static void rng_seed(PyRng* r, uint64_t seed) {
    uint32_t key[2];
    int klen = 1;
    key[0] = (uint32_t)seed;
    key[1] = (uint32_t)(seed >> 32);
    if (key[1]) klen = 2;
    rng_init_by_array(r, key, klen);
}

static uint32_t rng_u32(PyRng* r) {
    static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
    uint32_t y;
    if (r->mti >= MT_N) {
        int kk;
        for (kk = 0; kk < MT_N - MT_M; kk++) {
            y = (r->mt[kk] & 0x80000000U) | (r->mt[kk + 1] & 0x7fffffffU);
            r->mt[kk] = r->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1U];
        }
        for (; kk < MT_N - 1; kk++) {
            y = (r->mt[kk] & 0x80000000U) | (r->mt[kk + 1] & 0x7fffffffU);
            r->mt[kk] = r->mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1U];
        }
        y = (r->mt[MT_N - 1] & 0x80000000U) | (r->mt[0] & 0x7fffffffU);
        r->mt[MT_N - 1] = r->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1U];
        r->mti = 0;
    }
    y = r->mt[r->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

static double rng_random(PyRng* r) {
    uint32_t a = rng_u32(r) >> 5, b = rng_u32(r) >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

static uint32_t rng_below(PyRng* r, uint32_t n) {
    int k = 0;
    for (uint32_t t = n; t; t >>= 1) k++; /* n.bit_length() */
    uint32_t v = rng_u32(r) >> (32 - k);
    while (v >= n) v = rng_u32(r) >> (32 - k);
    return v;
}

static int rng_randint(PyRng* r, int a, int b) { return a + (int)rng_below(r, (uint32_t)(b - a + 1)); }

/* ------------------------------------------------------------------------ */
/* state                                                                     */
/* ------------------------------------------------------------------------ */
static const int DX[4] = {0, 1, 0, -1}; /* maze.py:19 DELTAS, N E S W */
static const int DY[4] = {-1, 0, 1, 0};

typedef struct {
    int x, y, dir, tag;
    int has_last_mark, lmx, lmy;
    int knows_end, sees_end, other_knows_end, has_key, sees_key, team_has_key;
    int exit_len;
    int route_len; /* -1 == None */
    int8_t route[ROUTE_CAP];
    int olsx, olsy;
    long long tfls;
    int mem[4];
    int minx, maxx, miny, maxy;
    int cur_t;
    int nme[4]; /* next_move_to_exit, maze_agent.py:113-118 */
} OAgent;

typedef struct {
    int w, h;
    uint8_t layout[41 * 41 + 64];
    int sx, sy, ex, ey;
    int key_valid, kx, ky;
    int path_len;
    int16_t path[41 * 41 + 64][2];
    int t;
    int error;
    PyRng rng;
    OAgent ag[2];
} OMaze;

typedef struct {
    int n;
    int size_w, size_h; /* default_size (cells) */
    int max_t, difficulty, rand_start, rand_sizes, lo, hi;
    OMaze* m;
} OEnv;

#define CELL(M, X, Y) ((M)->layout[(Y) * (M)->w + (X)])

static int in_bounds(const OMaze* m, int x, int y) { return x >= 0 && x < m->w && y >= 0 && y < m->h; } /* maze.py:166-167 */

/* ------------------------------------------------------------------------ */
/* maze generation: maze.py:170-273                                          */
/* ------------------------------------------------------------------------ */
static void set_start(const OEnv* e, OMaze* m) { /* maze.py:229-237 */
    if (e->rand_start) {
        m->sx = rng_randint(&m->rng, 0, (m->w - 1) / 2) * 2;
        m->sy = rng_randint(&m->rng, 0, (m->h - 1) / 2) * 2;
    } else {
        m->sx = ((m->w / 2) % 2 == 0) ? m->w / 2 : m->w / 2 - 1;
        m->sy = 0;
    }
}

static int set_end(OMaze* m) { /* maze.py:239-250 */
    int coin = rng_randint(&m->rng, 0, 1);
    int x = coin == 0 ? 0 : m->w - 1;
    for (long tries = 0; tries < GEN_TRIES; tries++) {
        int y = rng_randint(&m->rng, 0, m->h - 1);
        if (x == m->sx && y == m->sy) continue;
        if (CELL(m, x, y) == 0) { m->ex = x; m->ey = y; return 0; }
    }
    return -1;
}

/* Unique start->end path in the spanning tree (maze.py:261-273 DFS result). */
static int tree_path(const OMaze* m, int16_t (*out)[2]) {
    static int16_t par[41 * 41 + 64];
    static int16_t q[41 * 41 + 64];
    int n = m->w * m->h;
    for (int i = 0; i < n; i++) par[i] = -2;
    int head = 0, tail = 0, s = m->sy * m->w + m->sx, goal = m->ey * m->w + m->ex;
    q[tail++] = (int16_t)s;
    par[s] = -1;
    while (head < tail) {
        int c = q[head++];
        if (c == goal) break;
        int cx = c % m->w, cy = c / m->w;
        for (int d = 0; d < 4; d++) {
            int nx = cx + DX[d], ny = cy + DY[d];
            if (!in_bounds(m, nx, ny) || CELL(m, nx, ny) != 0) continue;
            int ni = ny * m->w + nx;
            if (par[ni] != -2) continue;
            par[ni] = (int16_t)c;
            q[tail++] = (int16_t)ni;
        }
    }
    int len = 0;
    for (int c = goal; c != -1; c = par[c]) len++;
    int k = len - 1;
    for (int c = goal; c != -1; c = par[c], k--) { out[k][0] = (int16_t)(c % m->w); out[k][1] = (int16_t)(c / m->w); }
    return len;
}

static int build_maze(const OEnv* e, OMaze* m) { /* maze.py:170-218 */
    if (e->rand_sizes) {
        int size = rng_randint(&m->rng, e->lo, e->hi) * 2 - 1;
        m->w = m->h = size;
    } else {
        m->w = e->size_w * 2 - 1;
        m->h = e->size_h * 2 - 1;
    }
    memset(m->layout, 1, (size_t)(m->w * m->h));
    set_start(e, m);
    /* recursive backtracker: maze.py:180-201 */
    static int16_t stk[41 * 41][2];
    int sp = 0;
    stk[sp][0] = (int16_t)m->sx;
    stk[sp][1] = (int16_t)m->sy;
    sp++;
    double corridor = 0.0;
    const double inc = 1.0 / (10 * (m->w > m->h ? m->w : m->h));
    while (sp) {
        int cx = stk[sp - 1][0], cy = stk[sp - 1][1];
        CELL(m, cx, cy) = 0;
        int nb[4][2], nn = 0;
        for (int d = 0; d < 4; d++) { /* get_neighbors maze.py:220-227 */
            int nx = cx + 2 * DX[d], ny = cy + 2 * DY[d];
            if (in_bounds(m, nx, ny) && CELL(m, nx, ny) == 1) { nb[nn][0] = nx; nb[nn][1] = ny; nn++; }
        }
        if (nn && rng_random(&m->rng) > corridor) {
            int pick = (int)rng_below(&m->rng, (uint32_t)nn);
            int nx = nb[pick][0], ny = nb[pick][1];
            CELL(m, (cx + nx) / 2, (cy + ny) / 2) = 0;
            stk[sp][0] = (int16_t)nx;
            stk[sp][1] = (int16_t)ny;
            sp++;
            corridor += inc;
        } else {
            sp--;
            corridor = 0.0;
        }
    }
    /* difficulty x (set_end + path); last end among the longest wins (maze.py:204-217) */
    int best_len = 0, bex = 0, bey = 0;
    for (int r = 0; r < e->difficulty; r++) {
        if (set_end(m)) { /* give up: end = start, path = [start], no key */
            m->ex = m->sx;
            m->ey = m->sy;
            m->path_len = 1;
            m->path[0][0] = (int16_t)m->sx;
            m->path[0][1] = (int16_t)m->sy;
            m->path[1][0] = (int16_t)m->sx;
            m->path[1][1] = (int16_t)m->sy;
            m->key_valid = 0;
            return -1;
        }
        int len = tree_path(m, m->path);
        if (len > best_len) best_len = len;
        if (len == best_len) { bex = m->ex; bey = m->ey; }
    }
    m->ex = bex;
    m->ey = bey;
    m->path_len = tree_path(m, m->path);
    /* set_key: maze.py:252-259 */
    m->key_valid = 0;
    for (long tries = 0;; tries++) {
        if (tries >= GEN_TRIES) return -1;
        int x = rng_randint(&m->rng, 0, m->w - 1);
        int y = rng_randint(&m->rng, 0, m->h - 1);
        if (CELL(m, x, y) == 1 || (x == m->ex && y == m->ey) || (x == m->sx && y == m->sy)) continue;
        int on_path = 0;
        for (int i = 0; i < m->path_len; i++)
            if (m->path[i][0] == x && m->path[i][1] == y) { on_path = 1; break; }
        if (on_path) continue;
        m->kx = x;
        m->ky = y;
        m->key_valid = 1;
        return 0;
    }
}

/* ------------------------------------------------------------------------ */
/* agent: maze_agent.py                                                      */
/* ------------------------------------------------------------------------ */
static void agent_init(OAgent* a, int tag) { /* maze_agent.py:16-57 */
    memset(a, 0, sizeof(*a));
    a->tag = tag;
    a->x = a->y = 0;
    a->dir = 2;
    a->exit_len = -1;
    a->route_len = -1;
    for (int i = 0; i < 4; i++) a->mem[i] = -1;
    a->minx = a->maxx = 0;
    a->miny = a->maxy = 0;
}

static void agent_reset(OAgent* a, int x, int y) { /* maze_agent.py:59-79 (tfls NOT reset) */
    a->cur_t = 0;
    a->x = x;
    a->y = y;
    a->olsx = x;
    a->olsy = y;
    a->minx = a->maxx = x; /* reset_estimates :338-344 */
    a->miny = a->maxy = y;
    a->dir = 2;
    a->has_last_mark = 0;
    for (int i = 0; i < 4; i++) a->mem[i] = -1;
    a->knows_end = a->other_knows_end = a->sees_end = 0;
    for (int i = 0; i < 4; i++) a->nme[i] = 0;
    a->exit_len = -1;
    a->route_len = -1;
    a->has_key = a->team_has_key = a->sees_key = 0;
}

static int is_open(const OMaze* m, int x, int y) { return in_bounds(m, x, y) && CELL(m, x, y) != 1; }

/* neighbours relative to facing: maze_agent.py:347-358 */
static void rel_neighbors(const OMaze* m, const OAgent* a, int x, int y, int out[4]) {
    for (int i = 0; i < 4; i++) {
        int d = (i + a->dir) % 4;
        out[i] = is_open(m, x + DX[d], y + DY[d]);
    }
}

static void route_copy(OAgent* dst, const OAgent* src) {
    dst->route_len = src->route_len < 0 ? 0 : src->route_len;
    if (src->route_len > 0) memcpy(dst->route, src->route, (size_t)src->route_len);
}

static int route_push(OAgent* a, int v, OMaze* m) {
    if (a->route_len < 0) a->route_len = 0;
    if (a->route_len >= ROUTE_CAP) { m->error |= 4; return -1; }
    a->route[a->route_len++] = (int8_t)v;
    return 0;
}

/* positions of the agents as seen by get_visibility_features (maze.agent_positions) */
typedef struct {
    int n;       /* number of agents registered */
    int idx[2];  /* agent indices */
} Positions;

/* get_visibility_features: maze_agent.py:188-277 */
static void visibility(OMaze* m, int self_i, const Positions* pos, double own_mark[4], double oth_mark[4],
                       int vis_agents[4], int vis_key[4], int vad[4], double other_rel[2]) {
    OAgent* s = &m->ag[self_i];
    OAgent* o = &m->ag[1 - self_i];
    int nva = 0;
    for (int i = 0; i < 4; i++) { own_mark[i] = oth_mark[i] = 0.0; vis_agents[i] = vis_key[i] = vad[i] = 0; }
    s->tfls += 1;
    s->sees_end = (s->x == m->ex && s->y == m->ey);
    s->sees_key = 0;
    /* co-location: :199-213 */
    if (o->x == s->x && o->y == s->y) {
        s->tfls = 0;
        for (int i = 0; i < 4 && nva < 4; i++) vis_agents[nva++] = 1;
        s->olsx = o->x;
        s->olsy = o->y;
        s->team_has_key = s->team_has_key || o->has_key;
        s->other_knows_end = s->other_knows_end || o->knows_end;
        vad[o->dir] = 1;
        if (s->knows_end && !o->knows_end) {
            route_copy(o, s);
            s->other_knows_end = 1;
            o->knows_end = 1;
            o->other_knows_end = 1;
        }
    }
    /* rays: :215-269 */
    for (int d = 0; d < 4; d++) {
        int ad = (d + s->dir) % 4;
        int nx = s->x, ny = s->y;
        for (int j = 1; j <= 4; j++) {
            nx += DX[ad];
            ny += DY[ad];
            if (!in_bounds(m, nx, ny) || CELL(m, nx, ny) == 1) break;
            if (nx == m->ex && ny == m->ey) {
                s->knows_end = 1;
                s->sees_end = 1;
                if (s->exit_len == -1) {
                    s->route_len = 0;
                    for (int k = 0; k < j; k++) s->route[s->route_len++] = (int8_t)ad;
                    s->exit_len = j;
                }
            }
            if (m->key_valid && nx == m->kx && ny == m->ky) {
                s->sees_key = 1;
                vis_key[d] = 1;
            }
            for (int p = 0; p < pos->n; p++) {
                int ai = pos->idx[p];
                OAgent* g = &m->ag[ai];
                if (ai == self_i || g->x != nx || g->y != ny) continue;
                s->tfls = 0;
                s->olsx = g->x;
                s->olsy = g->y;
                s->other_knows_end = s->other_knows_end || g->knows_end;
                s->team_has_key = s->team_has_key || g->has_key;
                vad[g->dir] = 1;
                if (nva + 4 <= 4) { vis_agents[d] = 1; nva += 4; } else m->error |= 8;
                if (j == 1 && s->knows_end && !g->knows_end) {
                    route_copy(g, s);
                    if (s->route_len > 0 && ad == s->route[s->route_len - 1]) g->route_len--;
                    else route_push(g, (ad + 2) % 4, m);
                    s->other_knows_end = 1;
                    g->knows_end = 1;
                    g->other_knows_end = 1;
                }
            }
            uint8_t c = CELL(m, nx, ny);
            if (c == s->tag) own_mark[d] += 1.0 / 4;
            else if (c > 1) oth_mark[d] += 1.0 / 4;
            /* update_maze_minmax :313-328 */
            if (ad == 0 && ny < s->miny) s->miny = ny;
            else if (ad == 1 && nx > s->maxx) s->maxx = nx;
            else if (ad == 2 && ny > s->maxy) s->maxy = ny;
            else if (ad == 3 && nx < s->minx) s->minx = nx;
        }
    }
    /* update_maze_dims :330-336 */
    int west = s->maxx - s->minx, hest = s->maxy - s->miny;
    if (west == 0) west = 1;
    if (hest == 0) hest = 1;
    other_rel[0] = (double)(s->olsx - s->minx) / west;
    other_rel[1] = (double)(s->maxy - s->olsy) / hest;
}

/* get_dead_ends: maze_agent.py:143-185 */
static void dead_ends(const OMaze* m, const OAgent* s, double de[4], int mmask[4]) {
    int nb[4];
    rel_neighbors(m, s, s->x, s->y, nb);
    for (int d = 0; d < 4; d++) { mmask[d] = nb[d]; de[d] = nb[d] ? 0.0 : 1.0; }
    for (int d = 0; d < 4; d++) {
        if (de[d] == 1.0) continue;
        int ad = (d + s->dir) % 4;
        int nx = s->x, ny = s->y;
        for (int j = 1; j <= 4; j++) {
            nx += DX[ad];
            ny += DY[ad];
            int n2[4];
            rel_neighbors(m, s, nx, ny, n2);
            if (n2[(d + 1) % 4] || n2[(d + 3) % 4]) break;
            int cnt = n2[0] + n2[1] + n2[2] + n2[3];
            if (cnt == 1) { de[d] = 1.0 - j * (1.0 / 4); break; }
            else if (!n2[d]) break;
        }
    }
    if (!s->sees_end && !s->sees_key)
        for (int d = 0; d < 4; d++) mmask[d] = (de[d] == 0.0);
}

/* get_observations: maze_agent.py:89-140 */
static void observe(OEnv* e, OMaze* m, int self_i, const Positions* pos, float* obs, uint8_t* mask) {
    OAgent* s = &m->ag[self_i];
    double own[4], oth[4], orel[2], de[4];
    int va[4], vk[4], vad[4], mm[4];
    visibility(m, self_i, pos, own, oth, va, vk, vad, orel);
    dead_ends(m, s, de, mm);
    double f[OBS_DIM];
    int k = 0;
    for (int i = 0; i < 4; i++) f[k++] = (i == s->dir);
    for (int i = 0; i < 4; i++) f[k++] = de[i];
    for (int i = 0; i < 4; i++) f[k++] = own[i];
    for (int i = 0; i < 4; i++) f[k++] = oth[i];
    for (int i = 0; i < 4; i++) f[k++] = va[i];
    for (int i = 0; i < 4; i++) f[k++] = vad[i];
    for (int i = 0; i < 4; i++) f[k++] = vk[i];
    for (int i = 0; i < 4; i++) /* get_memory :289-294 */
        for (int mv = 0; mv < 4; mv++) f[k++] = (s->mem[i] == mv);
    /* last mark direction: get_direction_from :297-311 */
    int lm[4] = {0, 0, 0, 0};
    if (s->has_last_mark) {
        if (s->lmx == s->x && s->lmy == s->y) { lm[0] = lm[1] = lm[2] = lm[3] = 1; }
        else {
            if (s->lmy > s->y) lm[(2 - s->dir + 4) % 4] = 1;
            else if (s->lmy < s->y) lm[(0 - s->dir + 4) % 4] = 1;
            if (s->lmx > s->x) lm[(1 - s->dir + 4) % 4] = 1;
            else if (s->lmx < s->x) lm[(3 - s->dir + 4) % 4] = 1;
        }
    }
    for (int i = 0; i < 4; i++) f[k++] = lm[i];
    int west = s->maxx - s->minx, hest = s->maxy - s->miny;
    if (west == 0) west = 1;
    if (hest == 0) hest = 1;
    f[k++] = (double)(s->x - s->minx) / west;
    f[k++] = (double)(s->maxy - s->y) / hest;
    f[k++] = orel[0];
    f[k++] = orel[1];
    f[k++] = s->sees_end;
    int nme[4] = {0, 0, 0, 0};
    if (s->route_len > 0) nme[(s->route[s->route_len - 1] - s->dir + 4) % 4] = 1;
    else nme[0] = nme[1] = nme[2] = nme[3] = 1;
    for (int i = 0; i < 4; i++) { s->nme[i] = nme[i]; f[k++] = nme[i]; }
    f[k++] = s->exit_len < 40 ? s->exit_len / 40.0 : 1.0;
    f[k++] = s->other_knows_end;
    f[k++] = s->has_key;
    f[k++] = s->team_has_key;
    f[k++] = s->tfls < 40 ? (double)s->tfls / 40.0 : 1.0;
    f[k++] = (double)s->cur_t / e->max_t;
    f[k++] = (s->tag == 2);
    f[k++] = (s->tag == 3);
    for (int i = 0; i < OBS_DIM; i++) obs[i] = (float)f[i];
    /* action mask :132-139 */
    if (vk[0] || vk[1] || vk[2] || vk[3]) {
        int first = vk[0] ? 0 : vk[1] ? 1 : vk[2] ? 2 : 3;
        for (int i = 0; i < 4; i++) mm[i] = (i == first);
    }
    int any_va = va[0] || va[1] || va[2] || va[3];
    for (int i = 0; i < 4; i++) mask[i] = (uint8_t)mm[i];
    mask[4] = (uint8_t)(any_va && s->x == m->ex && s->x == m->ey); /* Q2: (x, x) == end */
    mask[5] = (uint8_t)(CELL(m, s->x, s->y) != s->tag);
}

/* Maze.reset: maze.py:55-72 */
static int maze_reset(OEnv* e, OMaze* m, float* obs, uint8_t* masks) {
    m->t = 0;
    int rc = 0;
    if (build_maze(e, m)) { m->error |= 1; rc = -1; }
    Positions pos = {0, {0, 0}};
    for (int i = 0; i < 2; i++) {
        agent_reset(&m->ag[i], m->path[i][0], m->path[i][1]);
        pos.idx[pos.n++] = i;
        observe(e, m, i, &pos, obs + i * OBS_DIM, masks + i * MASK_DIM);
    }
    return rc;
}

/* single_agent_step: maze.py:124-163; returns got_key */
static int agent_step(OMaze* m, int i, int move, int mark) {
    OAgent* a = &m->ag[i];
    a->cur_t = m->t;
    int got = 0;
    if (mark == 1) {
        CELL(m, a->x, a->y) = (uint8_t)a->tag;
        a->has_last_mark = 1;
        a->lmx = a->x;
        a->lmy = a->y;
    }
    if (move != 4) {
        int d = (move + a->dir) % 4;
        int nx = a->x + DX[d], ny = a->y + DY[d];
        if (!is_open(m, nx, ny)) { m->error |= 2; return 0; } /* reference only prints (:141-145) */
        if (a->knows_end) {
            if (a->route_len > 0 && d == a->route[a->route_len - 1]) { a->route_len--; a->exit_len--; }
            else { route_push(a, (d + 2) % 4, m); a->exit_len++; }
        }
        a->x = nx;
        a->y = ny;
        a->dir = d;
        if (m->key_valid && nx == m->kx && ny == m->ky) {
            m->key_valid = 0;
            a->has_key = 1;
            a->team_has_key = 1;
            got = 1;
        }
        a->mem[0] = a->mem[1]; /* deque(maxlen=4).append */
        a->mem[1] = a->mem[2];
        a->mem[2] = a->mem[3];
        a->mem[3] = move;
    }
    return got;
}

/* Maze.step: maze.py:74-122 */
static void maze_step(OEnv* e, OMaze* m, const int8_t* act, float* obs, uint8_t* masks, float* reward,
                      uint8_t* done) {
    m->t += 1;
    int have_key = 0, first_key = 0;
    for (int i = 0; i < 2; i++) {
        first_key += agent_step(m, i, act[2 * i], act[2 * i + 1]);
        have_key += m->ag[i].has_key;
    }
    Positions pos = {2, {0, 1}};
    int exit_ready = 1;
    for (int i = 0; i < 2; i++) {
        observe(e, m, i, &pos, obs + i * OBS_DIM, masks + i * MASK_DIM);
        exit_ready = exit_ready && m->ag[i].team_has_key && m->ag[i].knows_end;
    }
    if (exit_ready) {
        for (int i = 0; i < 2; i++) {
            uint8_t* mk = masks + i * MASK_DIM;
            OAgent* a = &m->ag[i];
            if (!(a->x == m->ex && a->y == m->ey)) {
                int am = 0; /* np.argmax */
                for (int q = 1; q < 4; q++)
                    if (a->nme[q] > a->nme[am]) am = q;
                for (int q = 0; q < 4; q++) mk[q] = (uint8_t)(q == am);
            } else {
                mk[0] = mk[1] = mk[2] = mk[3] = 0;
                mk[4] = 1;
            }
        }
    }
    float r = (float)(first_key * 0.5);
    uint8_t dn = 0;
    int colocated = m->ag[0].x == m->ag[1].x && m->ag[0].y == m->ag[1].y;
    if (have_key && colocated && m->ag[0].x == m->ex && m->ag[0].y == m->ey) { r = 1.0f; dn = 1; }
    else if (m->t >= e->max_t) dn = 1;
    *reward = r;
    *done = dn;
}

/* ------------------------------------------------------------------------ */
/* exported API (ctypes)                                                     */
/* ------------------------------------------------------------------------ */
OEnv* oenv_new(int n, int size_w, int size_h, int max_t, int difficulty, int rand_start, int rand_sizes, int lo,
               int hi) {
    OEnv* e = (OEnv*)calloc(1, sizeof(OEnv));
    e->n = n;
    e->size_w = size_w;
    e->size_h = size_h;
    e->max_t = max_t;
    e->difficulty = difficulty;
    e->rand_start = rand_start;
    e->rand_sizes = rand_sizes;
    e->lo = lo;
    e->hi = hi;
    e->m = (OMaze*)calloc((size_t)n, sizeof(OMaze));
    for (int i = 0; i < n; i++) {
        agent_init(&e->m[i].ag[0], 2);
        agent_init(&e->m[i].ag[1], 3);
    }
    return e;
}

void oenv_free(OEnv* e) {
    if (!e) return;
    free(e->m);
    free(e);
}

void oenv_seed(OEnv* e, int i, uint64_t seed) { rng_seed(&e->m[i].rng, seed); }

void oenv_set_rng(OEnv* e, int i, const uint32_t* st625) {
    memcpy(e->m[i].rng.mt, st625, MT_N * 4);
    e->m[i].rng.mti = (int)st625[MT_N];
}

void oenv_get_rng(const OEnv* e, int i, uint32_t* st625) {
    memcpy(st625, e->m[i].rng.mt, MT_N * 4);
    st625[MT_N] = (uint32_t)e->m[i].rng.mti;
}

int oenv_reset(OEnv* e, int i, float* obs, uint8_t* masks) { return maze_reset(e, &e->m[i], obs, masks); }

void oenv_step(OEnv* e, int i, const int8_t* act, float* obs, uint8_t* masks, float* reward, uint8_t* done) {
    maze_step(e, &e->m[i], act, obs, masks, reward, done);
}

/* all mazes: act [n,2,2]; outputs [n,2,65], [n,2,6], [n], [n].  auto_reset
 * replaces obs/masks of finished mazes by their reset observation (PPO.py:127-130). */
int oenv_step_all(OEnv* e, const int8_t* act, float* obs, uint8_t* masks, float* reward, uint8_t* done,
                  int auto_reset) {
    int err = 0;
    for (int i = 0; i < e->n; i++) {
        maze_step(e, &e->m[i], act + 4 * i, obs + i * 2 * OBS_DIM, masks + i * 2 * MASK_DIM, reward + i, done + i);
        if (auto_reset && done[i])
            if (maze_reset(e, &e->m[i], obs + i * 2 * OBS_DIM, masks + i * 2 * MASK_DIM)) err = -1;
    }
    return err;
}

int oenv_reset_all(OEnv* e, float* obs, uint8_t* masks) {
    int err = 0;
    for (int i = 0; i < e->n; i++)
        if (maze_reset(e, &e->m[i], obs + i * 2 * OBS_DIM, masks + i * 2 * MASK_DIM)) err = -1;
    return err;
}

/* maze info: [w, h, sx, sy, ex, ey, key_valid, kx, ky, path_len, t, error] */
void oenv_get_maze(const OEnv* e, int i, int32_t* info, uint8_t* layout /* [h*w] */, int16_t* path /* [path_len,2] */) {
    const OMaze* m = &e->m[i];
    int32_t v[12] = {m->w, m->h, m->sx, m->sy, m->ex, m->ey, m->key_valid, m->kx, m->ky, m->path_len, m->t, m->error};
    memcpy(info, v, sizeof(v));
    if (layout) memcpy(layout, m->layout, (size_t)(m->w * m->h));
    if (path) memcpy(path, m->path, (size_t)m->path_len * 4);
}

/* per-agent state in the order of tests/golden/make_golden.py agent_state() */
void oenv_get_agent(const OEnv* e, int i, int ai, int32_t* out /* [25] */) {
    const OAgent* a = &e->m[i].ag[ai];
    int32_t v[25] = {a->x, a->y, a->dir, a->has_key, a->team_has_key, a->knows_end, a->other_knows_end,
                     a->exit_len, (int32_t)a->tfls, a->route_len,
                     a->route_len > 0 ? a->route[a->route_len - 1] : -1,
                     a->has_last_mark ? a->lmx : -1, a->has_last_mark ? a->lmy : -1,
                     a->minx, a->maxx, a->miny, a->maxy, a->olsx, a->olsy, a->sees_end, a->sees_key,
                     a->mem[0], a->mem[1], a->mem[2], a->mem[3]};
    memcpy(out, v, sizeof(v));
}

/* Direct access to the CPython RNG restatement (tests pin it against the stdlib). */
void orng_seed_stream(uint64_t seed, int n_words, uint32_t* out) {
    PyRng r;
    rng_seed(&r, seed);
    for (int i = 0; i < n_words; i++) out[i] = rng_u32(&r);
}

double orng_first_random(uint64_t seed) {
    PyRng r;
    rng_seed(&r, seed);
    return rng_random(&r);
}
