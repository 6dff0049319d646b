// env_device.h -- per-maze environment logic for gfx950 (device side).
//
// Restates, for one maze, Maze.step / single_agent_step (maze.py:74-163) and
// Agent.get_observations with its helpers (maze_agent.py:89-358).  Agents are
// processed strictly in order (agent 0 then agent 1), because agent 0's
// observation may rewrite agent 1's knowledge of the exit before agent 1
// observes (maze_agent.py:209-213, 252-260).
//
// Route representation: the reference keeps a per-agent stack of directions
// to the exit (maze.py:148-154).  The maze is a tree, every push/pop keeps
// that stack equal to the tree path from the agent's cell to the exit, and
// every copy between agents (maze_agent.py:210, 253-257) produces the
// receiver's tree path.  So the stack top is the per-cell "direction toward
// the exit" stored in bits 2-4 of the layout byte, the stack is empty exactly
// on the exit cell, and only the independent counter exit_len (Q6) is kept.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "marlmaze.h"

#ifndef MM_HD
#define MM_HD __host__ __device__ __forceinline__
#endif

namespace mm {

constexpr int kObs = MM_OBS_DIM;
constexpr int kMask = MM_MASK_DIM;
constexpr int kDirNone = 4;  // layout bits 2-4 on the exit cell

MM_HD int ddx(int d) { return (d == 1) - (d == 3); }  // maze.py:19 DELTAS
MM_HD int ddy(int d) { return (d == 2) - (d == 0); }

// Agent state in registers (mm_agent_t unpacked).
struct Agent {
    int x, y, dir, flags;
    int lmx, lmy, olsx, olsy;
    int minx, maxx, miny, maxy;
    uint32_t mem;  // byte i = slot i (0 = oldest), 0xff = -1
    int exit_len;
    int tfls;
    int tag;

    MM_HD bool f(int b) const { return (flags & b) != 0; }
    MM_HD void set(int b, bool v) { flags = v ? (flags | b) : (flags & ~b); }
};

MM_HD Agent load_agent(const mm_agent_t& a, int tag) {
    Agent r;
    r.x = a.x; r.y = a.y; r.dir = a.dir; r.flags = (uint8_t)a.flags;
    r.lmx = a.lmx; r.lmy = a.lmy; r.olsx = a.olsx; r.olsy = a.olsy;
    r.minx = a.minx; r.maxx = a.maxx; r.miny = a.miny; r.maxy = a.maxy;
    r.mem = (uint32_t)(uint8_t)a.mem[0] | ((uint32_t)(uint8_t)a.mem[1] << 8) |
            ((uint32_t)(uint8_t)a.mem[2] << 16) | ((uint32_t)(uint8_t)a.mem[3] << 24);
    r.exit_len = a.exit_len;
    r.tfls = a.tfls;
    r.tag = tag;
    return r;
}

MM_HD mm_agent_t pack_agent(const Agent& r) {
    mm_agent_t a;
    a.x = (int8_t)r.x; a.y = (int8_t)r.y; a.dir = (int8_t)r.dir; a.flags = (int8_t)r.flags;
    a.lmx = (int8_t)r.lmx; a.lmy = (int8_t)r.lmy; a.olsx = (int8_t)r.olsx; a.olsy = (int8_t)r.olsy;
    a.minx = (int8_t)r.minx; a.maxx = (int8_t)r.maxx; a.miny = (int8_t)r.miny; a.maxy = (int8_t)r.maxy;
    a.mem[0] = (int8_t)(r.mem & 0xff); a.mem[1] = (int8_t)((r.mem >> 8) & 0xff);
    a.mem[2] = (int8_t)((r.mem >> 16) & 0xff); a.mem[3] = (int8_t)(r.mem >> 24);
    a.exit_len = r.exit_len;
    a.tfls = r.tfls;
    a.reserved[0] = 0;
    a.reserved[1] = 0;
    return a;
}

// Agent.reset (maze_agent.py:59-79); time_from_last_seen is NOT reset (Q5).
MM_HD void reset_agent(Agent& a, int x, int y) {
    a.x = x; a.y = y;
    a.olsx = x; a.olsy = y;
    a.minx = a.maxx = x;  // reset_estimates :338-344
    a.miny = a.maxy = y;
    a.dir = 2;
    a.flags = 0;          // knows_end, sees_end, other_knows, has_key, sees_key, team_key, last mark
    a.lmx = a.lmy = 0;
    a.mem = 0xffffffffu;
    a.exit_len = -1;
}

// Read-only view of one maze.  L may point into LDS.
struct View {
    uint8_t* L;
    int w, h, ex, ey, kx, ky;  // kx < 0: key picked (maze.py:157-158)
    int t, max_t;

    MM_HD bool inb(int x, int y) const { return x >= 0 && x < w && y >= 0 && y < h; }
    MM_HD int type(int x, int y) const { return L[y * w + x] & 3; }
    MM_HD int tdir(int x, int y) const { return (L[y * w + x] >> 2) & 7; }
    MM_HD bool open(int x, int y) const { return inb(x, y) && type(x, y) != 1; }
    MM_HD bool is_end(int x, int y) const { return x == ex && y == ey; }
};

// Relative neighbour openness of cell (x,y) for an agent facing `dir`
// (Agent.get_neighbors, maze_agent.py:347-358): bit i = direction (i+dir)%4 open.
MM_HD int rel_nbrs(const View& v, int dir, int x, int y) {
    int r = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int d = (i + dir) & 3;
        r |= v.open(x + ddx(d), y + ddy(d)) ? (1 << i) : 0;
    }
    return r;
}

// One ray of the cross-shaped neighbourhood of (x, y) in absolute direction
// ad: every cell that the ray of get_visibility_features or the dead-end probe
// of get_dead_ends can touch, gathered with independent (clamped,
// unconditional) loads and kept as bitmasks.
struct DirWin {
    uint32_t fwd;    // bit j-1: cell j (1..5) along the ray is open (in bounds, not a wall)
    uint32_t side;   // bit j-1: a side neighbour ((ad+1) or (ad+3)) of ray cell j (1..4) is open
    uint32_t m2;     // bit j-1: ray cell j (1..4) holds a mark of tag 2
    uint32_t m3;     //                                    ... of tag 3
};

MM_HD DirWin gather_dir(const View& v, int x, int y, int ad) {
    const int dx = ddx(ad), dy = ddy(ad);
    const int sx = ddx((ad + 1) & 3), sy = ddy((ad + 1) & 3);  // right-hand side; left = -(sx, sy)
    // in-bounds cells along the ray, and whether each side row/column exists
    const int lim = dx > 0 ? v.w - 1 - x : (dx < 0 ? x : (dy > 0 ? v.h - 1 - y : y));
    const bool okr = (unsigned)(x + sx) < (unsigned)v.w && (unsigned)(y + sy) < (unsigned)v.h;
    const bool okl = (unsigned)(x - sx) < (unsigned)v.w && (unsigned)(y - sy) < (unsigned)v.h;
    const int step = dx + dy * v.w;
    const int offr = okr ? sx + sy * v.w : 0, offl = okl ? -(sx + sy * v.w) : 0;
    const int base = y * v.w + x;
    // all 13 cells are read unconditionally (clamped indices never leave the
    // maze; a missing side row reads the ray cell itself) and combined with
    // bitwise logic, so the reads issue back to back with no branches
    int c[5], cr[4], cl[4];
    int idx = base;
#pragma unroll
    for (int j = 1; j <= 5; j++) {
        idx += j <= lim ? step : 0;  // base + min(j, lim) * step, without multiplies
        c[j - 1] = v.L[idx] & 3;
        if (j <= 4) {
            cr[j - 1] = v.L[idx + offr] & 3;
            cl[j - 1] = v.L[idx + offl] & 3;
        }
    }
    DirWin w{0, 0, 0, 0};
#pragma unroll
    for (int j = 1; j <= 5; j++) {
        const uint32_t in = j <= lim;
        w.fwd |= (in & (uint32_t)(c[j - 1] != 1)) << (j - 1);
        if (j <= 4) {
            w.m2 |= (in & (uint32_t)(c[j - 1] == 2)) << (j - 1);
            w.m3 |= (in & (uint32_t)(c[j - 1] == 3)) << (j - 1);
            const uint32_t so = ((uint32_t)okr & (uint32_t)(cr[j - 1] != 1)) | ((uint32_t)okl & (uint32_t)(cl[j - 1] != 1));
            w.side |= (in & so) << (j - 1);
        }
    }
    return w;
}

// Distance j (1..L) at which the ray from (x, y) in absolute direction ad
// passes (tx, ty); 0 if it does not within the L visible cells.
MM_HD int ray_hit(int x, int y, int ad, int tx, int ty, int L) {
    // ad 1 (E, +x) and 3 (W, -x) are horizontal, 0 (N, -y) and 2 (S, +y)
    // vertical: (tx, ty) is on the ray iff its offset across the ray is 0 and
    // its distance along it is 1..L.  Selects, not integer multiplies, and
    // bitwise conditions (no divergent branches).
    const int rx = tx - x, ry = ty - y;
    const bool horiz = ad & 1;
    const int along = horiz ? rx : ry, across = horiz ? ry : rx;
    const int j = (ad == 1 || ad == 2) ? along : -along;
    return ((across == 0) & (j >= 1) & (j <= L)) ? j : 0;
}

// Geometry of one relative direction d of an observation, packed in a word:
// bits 0-2 L (visible cells), 3-5 j of the end, 6-8 j of the key, 9-11 j of
// the other agent (0 = not on this ray), 12-14 own marks, 15-17 other marks
// on the visible cells, 18-20 dead-end value in quarters (4 = wall next to
// the agent, 0..3 = 1 - j/4 with j=4 -> 0 (Q12)).  Depends only on the two
// positions, the facing and the layout -- never on the agents' knowledge --
// so it can be computed for both agents before the order-dependent replay.
MM_HD uint32_t summarize_dir(const View& v, int x, int y, int dir, int d, int tag, int qx, int qy, bool q_reg) {
    const int ad = (d + dir) & 3;
    const DirWin w = gather_dir(v, x, y, ad);
    const int t = __builtin_ctz(~w.fwd);
    const int L = t < 4 ? t : 4;
    const int je = ray_hit(x, y, ad, v.ex, v.ey, L);
    const int jk0 = ray_hit(x, y, ad, v.kx, v.ky, L), ja0 = ray_hit(x, y, ad, qx, qy, L);
    const int jk = (v.kx >= 0) ? jk0 : 0;
    const int ja = q_reg ? ja0 : 0;
    const uint32_t vis = (1u << L) - 1u;
    const int own = __builtin_popcount((tag == 2 ? w.m2 : w.m3) & vis);
    const int oth = __builtin_popcount((tag == 2 ? w.m3 : w.m2) & vis);
    // get_dead_ends (:150-181): walk j = 1..4 while cell j is open; a side
    // opening ends the walk (not a dead end), a closed cell j+1 makes cell j
    // a dead end at distance j.
    const uint32_t stop = (w.side | ~(w.fwd >> 1)) & 0xfu;
    const int j0 = __builtin_ctz(stop | 0x10u) + 1;  // 5: no stop within 4 cells
    const int dead = !(w.fwd & 1u) ? 4 : (((j0 <= 4) & !((w.side >> ((j0 - 1) & 31)) & 1u)) ? 4 - j0 : 0);
    return (uint32_t)L | (uint32_t)je << 3 | (uint32_t)jk << 6 | (uint32_t)ja << 9 | (uint32_t)own << 12 |
           (uint32_t)oth << 15 | (uint32_t)dead << 18;
}

MM_HD int sum_L(uint32_t s) { return s & 7; }
MM_HD int sum_je(uint32_t s) { return s >> 3 & 7; }
MM_HD int sum_jk(uint32_t s) { return s >> 6 & 7; }
MM_HD int sum_ja(uint32_t s) { return s >> 9 & 7; }
MM_HD int sum_own(uint32_t s) { return s >> 12 & 7; }
MM_HD int sum_oth(uint32_t s) { return s >> 15 & 7; }
MM_HD int sum_dead(uint32_t s) { return s >> 18 & 7; }

struct Vis {
    int va, vk, vad;  // visible agents / key per relative ray, other agent's facing (bitmasks)
};

// The order-dependent part of get_visibility_features (maze_agent.py:188-277):
// replays, from the four direction summaries, every state change the
// reference makes -- in its order (directions 0..3, cells in increasing j, a
// cell's end check before its agent check) -- on the observer s and on the
// other agent q.  Written with selects: the mazes of a wavefront take
// different paths, so branches would serialise.
MM_HD Vis replay(const View& v, Agent& s, Agent& q, const uint32_t sum[4]) {
    Vis r{0, 0, 0};
    int sf = s.flags, qf = q.flags;
    int tfls = s.tfls + 1;
    int olsx = s.olsx, olsy = s.olsy;
    int exit_len = s.exit_len;
    int minx = s.minx, maxx = s.maxx, miny = s.miny, maxy = s.maxy;
    bool sees_end = v.is_end(s.x, s.y);
    int vk = 0;
    const int share = ((qf & MM_AF_HAS_KEY) ? MM_AF_TEAM_KEY : 0) | ((qf & MM_AF_KNOWS_END) ? MM_AF_OTHER_KNOWS : 0);
    // co-location (:199-213); q's state may be stale (Q3).  The route copy
    // (implicit: tree path) marks both as knowing.
    const bool coloc = q.x == s.x && q.y == s.y;
    {
        const bool copy = coloc && (sf & MM_AF_KNOWS_END) && !(qf & MM_AF_KNOWS_END);
        tfls = coloc ? 0 : tfls;
        r.va = coloc ? 0xf : 0;
        r.vad = coloc ? 1 << q.dir : 0;
        olsx = coloc ? q.x : olsx;
        olsy = coloc ? q.y : olsy;
        sf |= coloc ? share : 0;
        sf |= copy ? MM_AF_OTHER_KNOWS : 0;
        qf |= copy ? (MM_AF_KNOWS_END | MM_AF_OTHER_KNOWS) : 0;
    }
#pragma unroll
    for (int d = 0; d < 4; d++) {  // rays (:215-269)
        const uint32_t sm = sum[d];
        const int L = sum_L(sm), je = sum_je(sm), jk = sum_jk(sm), ja = sum_ja(sm);
        // the other agent on this ray (:239-260); when it stands beyond the
        // end cell, the end check of this ray runs first
        const int known = (sf | ((je && !(ja && ja < je)) ? MM_AF_KNOWS_END : 0)) & MM_AF_KNOWS_END;
        const int shr = ((qf & MM_AF_HAS_KEY) ? MM_AF_TEAM_KEY : 0) | ((qf & MM_AF_KNOWS_END) ? MM_AF_OTHER_KNOWS : 0);
        const bool copy = ja == 1 && known && !(qf & MM_AF_KNOWS_END);
        tfls = ja ? 0 : tfls;
        olsx = ja ? q.x : olsx;
        olsy = ja ? q.y : olsy;
        sf |= ja ? shr : 0;
        r.vad |= ja ? 1 << q.dir : 0;
        r.va |= ja ? 1 << d : 0;
        sf |= copy ? MM_AF_OTHER_KNOWS : 0;
        qf |= copy ? (MM_AF_KNOWS_END | MM_AF_OTHER_KNOWS) : 0;
        // the end on this ray
        sf |= je ? MM_AF_KNOWS_END : 0;
        sees_end = sees_end || je;
        exit_len = (je && exit_len == -1) ? je : exit_len;  // route := [ad]*j == tree path
        vk |= jk ? 1 << d : 0;
        // update_maze_minmax (:313-328): the farthest visible cell decides
        const int ad = (d + s.dir) & 3;
        miny = (L && ad == 0) ? min(miny, s.y - L) : miny;
        maxx = (L && ad == 1) ? max(maxx, s.x + L) : maxx;
        maxy = (L && ad == 2) ? max(maxy, s.y + L) : maxy;
        minx = (L && ad == 3) ? min(minx, s.x - L) : minx;
    }
    sf = sees_end ? (sf | MM_AF_SEES_END) : (sf & ~MM_AF_SEES_END);
    sf = vk ? (sf | MM_AF_SEES_KEY) : (sf & ~MM_AF_SEES_KEY);
    s.flags = sf;
    q.flags = qf;
    s.tfls = tfls;
    s.olsx = olsx;
    s.olsy = olsy;
    s.exit_len = exit_len;
    s.minx = minx;
    s.maxx = maxx;
    s.miny = miny;
    s.maxy = maxy;
    r.vk = vk;
    return r;
}

// Observation vector (maze_agent.py:91-130) and action mask (:132-139) of s
// after its replay, computed unconditionally into o[65] / mk[6] (registers).
// Returns np.argmax(next_move_to_exit).
//
// The reference divides small Python ints in fp64 and the tensor holds the
// float32 of the quotient (PPO.py:144).  Both operands are integers below
// 2^24, exactly representable in f32, and 53 >= 2*24 + 2, so the correctly
// rounded f32 division gives the same float as fp64-then-round.
MM_HD int build_obs(const View& v, const Agent& s, const Vis& r, const uint32_t sum[4], float o[kObs],
                    uint8_t mk[kMask]) {
    int west = s.maxx - s.minx, hest = s.maxy - s.miny;  // update_maze_dims (:330-336)
    if (west == 0) west = 1;
    if (hest == 0) hest = 1;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        o[0 + i] = (i == s.dir) ? 1.f : 0.f;
        o[4 + i] = (float)sum_dead(sum[i]) * 0.25f;
        o[8 + i] = (float)sum_own(sum[i]) * 0.25f;
        o[12 + i] = (float)sum_oth(sum[i]) * 0.25f;
        o[16 + i] = (r.va >> i & 1) ? 1.f : 0.f;
        o[20 + i] = (r.vad >> i & 1) ? 1.f : 0.f;
        o[24 + i] = (r.vk >> i & 1) ? 1.f : 0.f;
    }
#pragma unroll
    for (int slot = 0; slot < 4; slot++) {  // get_memory (:289-294)
        const int mv = (int)(int8_t)((s.mem >> (8 * slot)) & 0xff);
#pragma unroll
        for (int k = 0; k < 4; k++) o[28 + 4 * slot + k] = (mv == k) ? 1.f : 0.f;
    }
    int lm = 0;  // get_direction_from (:297-311)
    if (s.f(MM_AF_HAS_MARK)) {
        if (s.lmx == s.x && s.lmy == s.y) {
            lm = 0xf;
        } else {
            if (s.lmy > s.y) lm |= 1 << ((2 - s.dir) & 3);
            else if (s.lmy < s.y) lm |= 1 << ((0 - s.dir) & 3);
            if (s.lmx > s.x) lm |= 1 << ((1 - s.dir) & 3);
            else if (s.lmx < s.x) lm |= 1 << ((3 - s.dir) & 3);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) o[44 + i] = (lm >> i & 1) ? 1.f : 0.f;
    o[48] = __fdiv_rn((float)(s.x - s.minx), (float)west);
    o[49] = __fdiv_rn((float)(s.maxy - s.y), (float)hest);
    o[50] = __fdiv_rn((float)(s.olsx - s.minx), (float)west);
    o[51] = __fdiv_rn((float)(s.maxy - s.olsy), (float)hest);
    o[52] = s.f(MM_AF_SEES_END) ? 1.f : 0.f;
    int nme_arg = 0, nme = 0xf;  // next_move_to_exit (:113-118)
    if (s.f(MM_AF_KNOWS_END) && !v.is_end(s.x, s.y)) {
        nme_arg = (v.tdir(s.x, s.y) - s.dir) & 3;
        nme = 1 << nme_arg;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) o[53 + i] = (nme >> i & 1) ? 1.f : 0.f;
    o[57] = s.exit_len < 40 ? __fdiv_rn((float)s.exit_len, 40.f) : 1.f;
    o[58] = s.f(MM_AF_OTHER_KNOWS) ? 1.f : 0.f;
    o[59] = s.f(MM_AF_HAS_KEY) ? 1.f : 0.f;
    o[60] = s.f(MM_AF_TEAM_KEY) ? 1.f : 0.f;
    o[61] = s.tfls < 40 ? __fdiv_rn((float)s.tfls, 40.f) : 1.f;
    o[62] = __fdiv_rn((float)v.t, (float)v.max_t);
    o[63] = s.tag == 2 ? 1.f : 0.f;
    o[64] = s.tag == 3 ? 1.f : 0.f;
    // action mask (:132-139)
    int nb = 0, mmask = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        nb |= (sum_dead(sum[d]) != 4) << d;  // open neighbour (get_neighbors, relative)
        mmask |= (sum_dead(sum[d]) == 0) << d;
    }
    if (s.f(MM_AF_SEES_END) || s.f(MM_AF_SEES_KEY)) mmask = nb;
    if (r.vk) mmask = r.vk & (-r.vk);  // one-hot at np.argmax(visible_key)
#pragma unroll
    for (int i = 0; i < 4; i++) mk[i] = (uint8_t)(mmask >> i & 1);
    mk[4] = (uint8_t)(r.va != 0 && s.x == v.ex && s.x == v.ey);  // (x, x) == end (Q2)
    mk[5] = (uint8_t)(v.type(s.x, s.y) != s.tag);
    return nme_arg;
}

// Agent.get_observations (maze_agent.py:89-140) incl. get_visibility_features
// (:188-277) and get_dead_ends (:143-185), one thread.  `s` is the observer,
// `q` the other agent; `q_registered` = q is in maze.agent_positions (false
// only for agent 0 inside Maze.reset, maze.py:64-71).  Returns
// np.argmax(next_move_to_exit).
template <typename OutF>
MM_HD int observe(const View& v, Agent& s, Agent& q, bool q_registered, OutF&& out, uint8_t* mk) {
    uint32_t sum[4];
#pragma unroll
    for (int d = 0; d < 4; d++) sum[d] = summarize_dir(v, s.x, s.y, s.dir, d, s.tag, q.x, q.y, q_registered);
    const Vis r = replay(v, s, q, sum);
    float o[kObs];
    uint8_t m[kMask];
    const int am = build_obs(v, s, r, sum, o, m);
#pragma unroll
    for (int i = 0; i < kObs; i++) out(i, o[i]);
#pragma unroll
    for (int i = 0; i < kMask; i++) mk[i] = m[i];
    return am;
}

// single_agent_step (maze.py:124-163).  Returns 1 if this agent picked up the
// key.  Marks are written to v.L and, if gl != nullptr, to global memory.
// An illegal move (into a wall / off the grid) is refused and flagged.
MM_HD int agent_step(View& v, Agent& a, int move, int mark, uint8_t* gl, uint32_t& status) {
    int got = 0;
    if (mark == 1) {
        const int idx = a.y * v.w + a.x;
        const uint8_t b = (uint8_t)((v.L[idx] & ~3) | a.tag);
        v.L[idx] = b;
        if (gl) __builtin_nontemporal_store(b, gl + idx);  // streaming: no dirty line left for the end-of-kernel release
        a.lmx = a.x;
        a.lmy = a.y;
        a.flags |= MM_AF_HAS_MARK;
    }
    if (move != 4) {
        if (move < 0 || move > 4) {
            status |= MM_ST_BAD_MOVE;
            return 0;
        }
        const int d = (move + a.dir) & 3;
        const int nx = a.x + ddx(d), ny = a.y + ddy(d);
        if (!v.open(nx, ny)) {  // reference prints and walks on (maze.py:141-145)
            status |= MM_ST_BAD_MOVE;
            return 0;
        }
        if (a.f(MM_AF_KNOWS_END)) {  // :148-154
            const int top = v.tdir(a.x, a.y);
            if (top != kDirNone && d == top) a.exit_len -= 1;
            else a.exit_len += 1;
        }
        a.x = nx;
        a.y = ny;
        a.dir = d;
        if (nx == v.kx && ny == v.ky) {
            v.kx = -1;
            v.ky = -1;
            a.flags |= MM_AF_HAS_KEY | MM_AF_TEAM_KEY;
            got = 1;
        }
        a.mem = (a.mem >> 8) | ((uint32_t)move << 24);  // deque(maxlen=4).append(move)
    }
    return got;
}

}  // namespace mm
