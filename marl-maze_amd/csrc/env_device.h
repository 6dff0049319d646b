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

// Agent.get_observations (maze_agent.py:89-140) incl. get_visibility_features
// (:188-277) and get_dead_ends (:143-185).  `s` is the observer, `q` the other
// agent; `q_registered` = q is in maze.agent_positions (false only for agent
// 0 inside Maze.reset, maze.py:64-71).  Writes 65 floats to o[] (stride
// ostride) and 6 mask bytes to mk[].  Returns np.argmax(next_move_to_exit).
template <typename OutF>
MM_HD int observe(const View& v, Agent& s, Agent& q, bool q_registered, OutF&& out,
                                       uint8_t* mk) {
    // --- get_visibility_features
    s.tfls += 1;
    bool sees_end = v.is_end(s.x, s.y);
    bool sees_key = false;
    int va = 0, vk = 0, vad = 0;
    int own[4] = {0, 0, 0, 0}, oth[4] = {0, 0, 0, 0};
    if (q.x == s.x && q.y == s.y) {  // co-location (:199-213), q's state may be stale (Q3)
        s.tfls = 0;
        va = 0xf;
        s.olsx = q.x; s.olsy = q.y;
        if (q.f(MM_AF_HAS_KEY)) s.flags |= MM_AF_TEAM_KEY;
        if (q.f(MM_AF_KNOWS_END)) s.flags |= MM_AF_OTHER_KNOWS;
        vad |= 1 << q.dir;
        if (s.f(MM_AF_KNOWS_END) && !q.f(MM_AF_KNOWS_END)) {  // route copy (implicit: tree path)
            s.flags |= MM_AF_OTHER_KNOWS;
            q.flags |= MM_AF_KNOWS_END | MM_AF_OTHER_KNOWS;
        }
    }
#pragma unroll
    for (int d = 0; d < 4; d++) {  // rays (:215-269)
        const int ad = (d + s.dir) & 3;
        const int dx = ddx(ad), dy = ddy(ad);
        int nx = s.x, ny = s.y;
#pragma unroll
        for (int j = 1; j <= 4; j++) {
            nx += dx;
            ny += dy;
            if (!v.inb(nx, ny)) break;
            const int c = v.type(nx, ny);
            if (c == 1) break;
            if (v.is_end(nx, ny)) {
                s.flags |= MM_AF_KNOWS_END;
                sees_end = true;
                if (s.exit_len == -1) s.exit_len = j;  // route := [ad]*j == tree path
            }
            if (nx == v.kx && ny == v.ky) {
                sees_key = true;
                vk |= 1 << d;
            }
            if (q_registered && q.x == nx && q.y == ny) {
                s.tfls = 0;
                s.olsx = q.x; s.olsy = q.y;
                if (q.f(MM_AF_KNOWS_END)) s.flags |= MM_AF_OTHER_KNOWS;
                if (q.f(MM_AF_HAS_KEY)) s.flags |= MM_AF_TEAM_KEY;
                vad |= 1 << q.dir;
                va |= 1 << d;
                if (j == 1 && s.f(MM_AF_KNOWS_END) && !q.f(MM_AF_KNOWS_END)) {
                    s.flags |= MM_AF_OTHER_KNOWS;  // copy + push/pop (:253-257) == tree path
                    q.flags |= MM_AF_KNOWS_END | MM_AF_OTHER_KNOWS;
                }
            }
            if (c == s.tag) own[d]++;
            else if (c > 1) oth[d]++;
            // update_maze_minmax (:313-328)
            if (ad == 0 && ny < s.miny) s.miny = ny;
            else if (ad == 1 && nx > s.maxx) s.maxx = nx;
            else if (ad == 2 && ny > s.maxy) s.maxy = ny;
            else if (ad == 3 && nx < s.minx) s.minx = nx;
        }
    }
    s.set(MM_AF_SEES_END, sees_end);
    s.set(MM_AF_SEES_KEY, sees_key);
    int west = s.maxx - s.minx, hest = s.maxy - s.miny;  // update_maze_dims (:330-336)
    if (west == 0) west = 1;
    if (hest == 0) hest = 1;

    // --- get_dead_ends
    const int nb = rel_nbrs(v, s.dir, s.x, s.y);
    int dead_q[4];  // dead-end value in quarters: 4 = wall, 0..3 = 1 - j/4 (j=4 -> 0, Q12)
    int mmask = nb;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        dead_q[d] = (nb >> d & 1) ? 0 : 4;
        if (!(nb >> d & 1)) continue;
        const int ad = (d + s.dir) & 3;
        const int dx = ddx(ad), dy = ddy(ad);
        int nx = s.x, ny = s.y;
#pragma unroll
        for (int j = 1; j <= 4; j++) {
            nx += dx;
            ny += dy;
            const int n2 = rel_nbrs(v, s.dir, nx, ny);
            if ((n2 >> ((d + 1) & 3) & 1) || (n2 >> ((d + 3) & 3) & 1)) break;
            if (__builtin_popcount((unsigned)n2) == 1) {
                dead_q[d] = 4 - j;
                break;
            } else if (!(n2 >> d & 1)) {
                break;
            }
        }
    }
    if (!sees_end && !sees_key) {
        mmask = 0;
#pragma unroll
        for (int d = 0; d < 4; d++) mmask |= (dead_q[d] == 0) ? (1 << d) : 0;
    }

    // --- observation vector (:91-130)
#pragma unroll
    for (int i = 0; i < 4; i++) out(0 + i, (i == s.dir) ? 1.f : 0.f);
#pragma unroll
    for (int i = 0; i < 4; i++) out(4 + i, (float)dead_q[i] * 0.25f);
#pragma unroll
    for (int i = 0; i < 4; i++) out(8 + i, (float)own[i] * 0.25f);
#pragma unroll
    for (int i = 0; i < 4; i++) out(12 + i, (float)oth[i] * 0.25f);
#pragma unroll
    for (int i = 0; i < 4; i++) out(16 + i, (va >> i & 1) ? 1.f : 0.f);
#pragma unroll
    for (int i = 0; i < 4; i++) out(20 + i, (vad >> i & 1) ? 1.f : 0.f);
#pragma unroll
    for (int i = 0; i < 4; i++) out(24 + i, (vk >> i & 1) ? 1.f : 0.f);
#pragma unroll
    for (int slot = 0; slot < 4; slot++) {  // get_memory (:289-294)
        const int mv = (int)(int8_t)((s.mem >> (8 * slot)) & 0xff);
#pragma unroll
        for (int k = 0; k < 4; k++) out(28 + 4 * slot + k, (mv == k) ? 1.f : 0.f);
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
    for (int i = 0; i < 4; i++) out(44 + i, (lm >> i & 1) ? 1.f : 0.f);
    // Python true division of ints in fp64, then float32 (PPO.py:144)
    out(48, (float)((double)(s.x - s.minx) / (double)west));
    out(49, (float)((double)(s.maxy - s.y) / (double)hest));
    out(50, (float)((double)(s.olsx - s.minx) / (double)west));
    out(51, (float)((double)(s.maxy - s.olsy) / (double)hest));
    out(52, sees_end ? 1.f : 0.f);
    int nme_arg = 0, nme = 0xf;  // next_move_to_exit (:113-118)
    if (s.f(MM_AF_KNOWS_END) && !v.is_end(s.x, s.y)) {
        nme_arg = (v.tdir(s.x, s.y) - s.dir) & 3;
        nme = 1 << nme_arg;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) out(53 + i, (nme >> i & 1) ? 1.f : 0.f);
    out(57, s.exit_len < 40 ? (float)((double)s.exit_len / 40.0) : 1.f);
    out(58, s.f(MM_AF_OTHER_KNOWS) ? 1.f : 0.f);
    out(59, s.f(MM_AF_HAS_KEY) ? 1.f : 0.f);
    out(60, s.f(MM_AF_TEAM_KEY) ? 1.f : 0.f);
    out(61, s.tfls < 40 ? (float)((double)s.tfls / 40.0) : 1.f);
    out(62, (float)((double)v.t / (double)v.max_t));
    out(63, s.tag == 2 ? 1.f : 0.f);
    out(64, s.tag == 3 ? 1.f : 0.f);

    // --- action mask (:132-139)
    if (vk) mmask = vk & (-vk);  // one-hot at np.argmax(visible_key)
#pragma unroll
    for (int i = 0; i < 4; i++) mk[i] = (uint8_t)(mmask >> i & 1);
    mk[4] = (uint8_t)(va != 0 && s.x == v.ex && s.x == v.ey);  // (x, x) == end (Q2)
    mk[5] = (uint8_t)(v.type(s.x, s.y) != s.tag);
    return nme_arg;
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
        if (gl) gl[idx] = b;
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
