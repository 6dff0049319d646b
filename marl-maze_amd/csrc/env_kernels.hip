// env_kernels.hip -- batched MARL-Maze environment on MI355X (gfx950).
//
// Kernels
//   k_seed   one thread per maze: random.seed(seed_i) into the maze's
//            CPython MT19937 row, Agent.__init__ state (maze_agent.py:24-57).
//   k_reset  one 64-lane wavefront per maze: Maze.build_maze (maze.py:170-259):
//            recursive-backtracker generation with the maze's own MT19937
//            stream in LDS, plus the per-cell direction-to-exit table.
//   k_reset_obs  one thread per reset maze: agent resets and the two reset
//            observations in the reference's order (maze.py:64-71: agent 0
//            observes while agent 1 still holds its previous state, Q3).
//   k_step   four lanes per maze, 32 mazes per workgroup: Maze.step()
//            (maze.py:74-122).  The workgroup's 32 layouts are one contiguous
//            HBM range, staged into LDS with 16-byte coalesced loads; each
//            lane gathers two rays of one agent's neighbourhood as bitmasks.
//            Finished mazes are appended to a done list that k_reset consumes
//            (PPO.py:127-130).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "env_device.h"
#include "marlmaze.h"
#include "mt19937_wave.h"

extern "C" int mm_layout_stride(int size_w, int size_h, int rand_sizes, int rand_lo, int rand_hi);

namespace mm {

constexpr int kMaxCells = MM_MAX_SIDE * MM_MAX_SIDE;
constexpr int kGenTries = 1 << 16;  // rejection-loop bound, same as oracle GEN_TRIES (reference: unbounded)
constexpr int kListOff = 64;        // done list starts at work[64]

// ---------------------------------------------------------------------------
// cooperative contiguous copies (whole workgroup)
// ---------------------------------------------------------------------------
// HBM -> LDS by LDS-DMA (16 bytes per lane, lane-linear): every piece is in
// flight at once and the copy waits once, at the caller's barrier (a
// register round trip per piece waited one HBM latency per loop iteration).
// src and dst 16-byte aligned.
__device__ __forceinline__ void copy_in(uint8_t* dst, const uint8_t* src, int bytes) {
    const int nv = bytes >> 4;
    const int lane = threadIdx.x & 63;
    const int wbase = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63);
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    for (int k0 = 0; k0 < nv; k0 += blockDim.x) {
        if (k0 + wbase + lane < nv)
            __builtin_amdgcn_global_load_lds(s4 + k0 + wbase + lane, dst + 16 * (k0 + wbase), 16, 0, 0);
    }
    for (int k = (nv << 4) + threadIdx.x; k < bytes; k += blockDim.x) dst[k] = src[k];
}

// Non-temporal (streaming) stores: the rows go out to memory while other
// workgroups still compute, instead of collecting as dirty L2 lines that the
// end-of-kernel release has to write back (k_step writes ~41 MB per launch at
// 65,536 mazes, more than the 32 MB of L2).
__device__ __forceinline__ void copy_out(uint8_t* dst, const uint8_t* src, int bytes) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int nv = bytes >> 4;
    const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
    u32x4* d4 = reinterpret_cast<u32x4*>(dst);
    for (int k = threadIdx.x; k < nv; k += blockDim.x) __builtin_nontemporal_store(s4[k], d4 + k);
    for (int k = (nv << 4) + threadIdx.x; k < bytes; k += blockDim.x) __builtin_nontemporal_store(src[k], dst + k);
}

// one 32-byte state record (mm_maze_t / mm_agent_t) as two streaming 16-byte stores
template <class T>
__device__ __forceinline__ void store_nt32(T* dst, const T& v) {
    static_assert(sizeof(T) == 32, "32-byte records");
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 w[2];
    __builtin_memcpy(w, &v, 32);
    __builtin_nontemporal_store(w[0], reinterpret_cast<u32x4*>(dst));
    __builtin_nontemporal_store(w[1], reinterpret_cast<u32x4*>(dst) + 1);
}

// ---------------------------------------------------------------------------
// seed
// ---------------------------------------------------------------------------
__global__ void k_seed(mm_env_t env, const uint64_t* __restrict__ seeds) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= env.n) return;
    mt_seed_thread(env.rng + (size_t)m * MM_RNG_WORDS, seeds[m]);
    for (int a = 0; a < 2; a++) {  // Agent.__init__ (maze_agent.py:24-57)
        Agent g;
        g.x = g.y = 0;
        g.dir = 2;
        g.flags = 0;
        g.lmx = g.lmy = 0;
        g.olsx = g.olsy = 0;
        g.minx = g.maxx = g.miny = g.maxy = 0;
        g.mem = 0xffffffffu;
        g.exit_len = -1;
        g.tfls = 0;
        g.tag = 2 + a;
        env.agents[2 * m + a] = pack_agent(g);
    }
    mm_maze_t z = {};
    z.kx = z.ky = -1;
    env.mazes[m] = z;
    if (env.gen_state) env.gen_state[m] = 1;  // a new stream: any pre-generated next maze is stale
}

// ---------------------------------------------------------------------------
// generation + reset (one wavefront per maze)
// ---------------------------------------------------------------------------
struct GenLds {
    uint32_t mt[kMtN];
    uint8_t cell[kMaxCells];     // layout being built (values 0/1)
    uint8_t par[kMaxCells];      // direction toward the root (start); bit 7 = on start->end path
    uint8_t pdir[kMaxCells];     // on-path cells: direction toward the end
    int16_t depth[kMaxCells];    // tree depth from start
    int16_t stack[kMaxCells];    // DFS stack (cell indices)
    int claim;                   // pre-generation protocol: the state lane 0 found / claimed
};

// Maze.build_maze + set_start/end/key (maze.py:170-259), wave-uniform.
// Returns false if a rejection loop exhausted its bound (the reference would
// loop forever).
__device__ bool generate(const mm_env_t& env, GenLds& g, WaveRng& rng, int& w, int& h, int& sx, int& sy, int& ex,
                         int& ey, int& kx, int& ky, int& plen, int& p1x, int& p1y) {
    const int lane = threadIdx.x;
    if (env.rand_sizes) {  // :171-174
        const int s = rng.randint(env.rand_lo, env.rand_hi) * 2 - 1;
        w = h = s;
    } else {
        w = env.size_w * 2 - 1;
        h = env.size_h * 2 - 1;
    }
    const int nc = w * h;
    for (int c = lane; c < nc; c += 64) {
        g.cell[c] = 1;
        g.par[c] = 0x7f;
        g.depth[c] = 0;
    }
    if (env.rand_start) {  // set_start :229-237
        sx = rng.randint(0, (w - 1) / 2) * 2;
        sy = rng.randint(0, (h - 1) / 2) * 2;
    } else {
        sx = ((w / 2) % 2 == 0) ? w / 2 : w / 2 - 1;
        sy = 0;
    }
    __syncthreads();
    // recursive backtracker :180-201
    int sp = 0;
    const int s0 = sy * w + sx;
    if (lane == 0) {
        g.stack[0] = (int16_t)s0;
        g.par[s0] = kDirNone;
    }
    sp = 1;
    double corridor = 0.0;
    const double inc = 1.0 / (10 * (w > h ? w : h));
    __syncthreads();
    while (sp > 0) {
        const int c = g.stack[sp - 1];
        const int cx = c % w, cy = c / w;
        int nbd[4] = {0, 0, 0, 0};
        int nn = 0;
#pragma unroll
        for (int d = 0; d < 4; d++) {  // get_neighbors :220-227
            const int nx = cx + 2 * ddx(d), ny = cy + 2 * ddy(d);
            if (nx >= 0 && nx < w && ny >= 0 && ny < h && g.cell[ny * w + nx] == 1) nbd[nn++] = d;
        }
        // layout[cur] = 0 (cells are only ever carved, so writing after the
        // neighbour scan is equivalent: the scan never looks at `c` itself)
        if (lane == 0) g.cell[c] = 0;
        if (nn && rng.random() > corridor) {
            const int pick = rng.below((uint32_t)nn);
            int d = nbd[0];
#pragma unroll
            for (int q = 1; q < 4; q++)
                if (q == pick) d = nbd[q];
            const int mx = cx + ddx(d), my = cy + ddy(d);
            const int nx = mx + ddx(d), ny = my + ddy(d);
            const int mi = my * w + mx, ni = ny * w + nx;
            const int back = (d + 2) & 3;
            if (lane == 0) {
                g.cell[mi] = 0;
                g.par[mi] = (uint8_t)back;
                g.par[ni] = (uint8_t)back;
                g.depth[mi] = (int16_t)(g.depth[c] + 1);
                g.depth[ni] = (int16_t)(g.depth[c] + 2);
                g.stack[sp] = (int16_t)ni;
            }
            sp++;
            corridor += inc;
        } else {
            sp--;
            corridor = 0.0;
        }
        __syncthreads();
    }
    // ends: difficulty x set_end, keep the longest (last of equal length) :204-217
    int best = 0;
    ex = ey = 0;
    for (int r = 0; r < env.difficulty; r++) {
        const int coin = rng.randint(0, 1);  // set_end :239-250
        const int x = coin == 0 ? 0 : w - 1;
        int y = -1;
        for (int tries = 0; tries < kGenTries; tries++) {
            const int yy = rng.randint(0, h - 1);
            if (x == sx && yy == sy) continue;
            if (g.cell[yy * w + x] == 0) {
                y = yy;
                break;
            }
        }
        if (y < 0) {  // give up (the reference loops forever): end = start, path = [start], no key
            ex = sx;
            ey = sy;
            plen = 1;
            p1x = sx;
            p1y = sy;
            kx = ky = -1;
            return false;
        }
        const int len = g.depth[y * w + x] + 1;  // len(get_shortest_path) in a tree
        if (len > best) best = len;
        if (len == best) {
            ex = x;
            ey = y;
        }
    }
    plen = best;
    // walk end -> start: mark the path, record the direction toward the end
    {
        int c = ey * w + ex;
        int prev = -1;
        p1x = ex;
        p1y = ey;
        while (true) {
            const uint8_t pd = g.par[c] & 0x7f;
            if (lane == 0) {
                g.par[c] = (uint8_t)(pd | 0x80);
                if (prev >= 0) {
                    // direction from c to prev = opposite of prev's parent direction
                    g.pdir[c] = (uint8_t)(((g.par[prev] & 0x7f) + 2) & 3);
                } else {
                    g.pdir[c] = kDirNone;
                }
            }
            if (pd == kDirNone) break;  // reached the start
            const int cx = c % w, cy = c / w;
            const int nx = cx + ddx(pd), ny = cy + ddy(pd);
            const int nxt = ny * w + nx;
            if (nxt == s0) {
                p1x = cx;
                p1y = cy;
            }
            prev = c;
            c = nxt;
            __syncthreads();
        }
    }
    __syncthreads();
    // set_key :252-259
    kx = ky = -1;
    for (int tries = 0; tries < kGenTries; tries++) {
        const int x = rng.randint(0, w - 1);
        const int y = rng.randint(0, h - 1);
        const int c = y * w + x;
        if (g.cell[c] == 1 || (x == ex && y == ey) || (x == sx && y == sy) || (g.par[c] & 0x80)) continue;
        kx = x;
        ky = y;
        break;
    }
    return kx >= 0;
}

// One maze generation from the MT state rs_in (624 words + index) into the
// layout row gl, the MT state after it into rs_out (may equal rs_in) and the
// generation fields of hdr: for the current maze (next = false) the maze's
// record is updated in place (t = 0, episode counters kept); for a
// pre-generated next maze (next = true) hdr is written fresh.
__device__ void generate_into(const mm_env_t& env, GenLds& g, const uint32_t* rs_in, uint32_t* rs_out, uint8_t* gl,
                              mm_maze_t* hdr, bool next) {
    const int lane = threadIdx.x;
    {  // the 624 state words: all loads in flight before the LDS writes
        constexpr int kPer = (kMtN + 63) / 64;
        uint32_t t[kPer];
#pragma unroll
        for (int u = 0; u < kPer; u++) t[u] = lane + 64 * u < kMtN ? rs_in[lane + 64 * u] : 0u;
#pragma unroll
        for (int u = 0; u < kPer; u++)
            if (lane + 64 * u < kMtN) g.mt[lane + 64 * u] = t[u];
    }
    WaveRng rng;
    rng.mt = g.mt;
    rng.idx = (int)rs_in[kMtN];
    rng.lane = lane;
    __syncthreads();
    int w, h, sx, sy, ex, ey, kx, ky, plen, p1x, p1y;
    const bool ok = generate(env, g, rng, w, h, sx, sy, ex, ey, kx, ky, plen, p1x, p1y);
    __syncthreads();
    // final layout bytes: cell | dir-to-exit << 2
    const int nc = w * h;
    for (int c = lane; c < nc; c += 64) {
        uint8_t b = g.cell[c];
        if (b == 0) {
            const uint8_t p = g.par[c];
            const int d = (p & 0x80) ? g.pdir[c] : (p & 0x7f);
            b = (uint8_t)(b | (d << 2));
        }
        gl[c] = b;
    }
    for (int k = lane; k < kMtN; k += 64) rs_out[k] = g.mt[k];
    if (lane == 0) rs_out[kMtN] = (uint32_t)rng.idx;
    __syncthreads();
    if (lane == 0) {
        mm_maze_t mz = {};
        if (!next) mz = *hdr;
        mz.t = 0;
        mz.w = (int8_t)w; mz.h = (int8_t)h;
        mz.ex = (int8_t)ex; mz.ey = (int8_t)ey;
        mz.kx = (int8_t)kx; mz.ky = (int8_t)ky;
        mz.sx = (int8_t)sx; mz.sy = (int8_t)sy;
        mz.path_len = (int16_t)plen;
        mz.spawn1 = p1x | (p1y << 8);  // second cell of the shortest path (agent 1's spawn)
        if (!ok) mz.status |= MM_ST_GEN_FAIL;
        *hdr = mz;
    }
}

__device__ __forceinline__ void generate_one(const mm_env_t& env, GenLds& g, int m) {
    uint32_t* rs = env.rng + (size_t)m * MM_RNG_WORDS;
    generate_into(env, g, rs, rs, env.layout + (size_t)m * env.layout_stride, env.mazes + m, false);
}

// ---------------------------------------------------------------------------
// pre-generation protocol (gen_state, see marlmaze.h)
// ---------------------------------------------------------------------------
enum { kGenReady = 0, kGenPending = 1, kGenRunning = 2, kGenInline = 3 };

__device__ __forceinline__ int gs_load(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gs_store(int32_t* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool gs_cas(int32_t* p, int expect, int v) {
    return __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                __HIP_MEMORY_SCOPE_AGENT);
}

// Maze.reset()'s generation for maze m (one wavefront): the pre-generated
// next maze copied in when it is ready, else generated inline (claimed so a
// concurrent mm_env_pregen leaves it alone); a next maze still being
// generated on the other stream is waited for.  Afterwards the maze's next
// maze is pending again.
__device__ void reset_one(const mm_env_t& env, GenLds& g, int m) {
    if (!env.gen_state) {
        generate_one(env, g, m);
        return;
    }
    const int lane = threadIdx.x;
    int32_t* st = env.gen_state + m;
    if (lane == 0) {
        int v;
        while (true) {
            v = gs_load(st);
            if (v == kGenReady) break;
            if (v == kGenPending && gs_cas(st, kGenPending, kGenInline)) {
                v = kGenInline;
                break;
            }
            __builtin_amdgcn_s_sleep(8);  // kGenRunning: the pre-generation in flight finishes by itself
        }
        g.claim = v;
    }
    __syncthreads();
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // every lane reads what the pre-generation released
    if (g.claim == kGenReady) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const int nv = env.layout_stride >> 4;  // layout_stride % 16 handled below
        const u32x4* src = reinterpret_cast<const u32x4*>(env.next_layout + (size_t)m * env.layout_stride);
        uint8_t* dst = env.layout + (size_t)m * env.layout_stride;
        if ((env.layout_stride & 15) == 0) {
            for (int k = lane; k < nv; k += 64) reinterpret_cast<u32x4*>(dst)[k] = src[k];
        } else {
            const uint8_t* sb = env.next_layout + (size_t)m * env.layout_stride;
            for (int k = lane; k < env.layout_stride; k += 64) dst[k] = sb[k];
        }
        const uint32_t* rn = env.next_rng + (size_t)m * MM_RNG_WORDS;
        uint32_t* rc = env.rng + (size_t)m * MM_RNG_WORDS;
        for (int k = lane; k < MM_RNG_WORDS; k += 64) rc[k] = rn[k];
        if (lane == 0) {
            const mm_maze_t nx = env.next_mazes[m];
            mm_maze_t mz = env.mazes[m];
            mz.t = 0;
            mz.w = nx.w; mz.h = nx.h;
            mz.ex = nx.ex; mz.ey = nx.ey;
            mz.kx = nx.kx; mz.ky = nx.ky;
            mz.sx = nx.sx; mz.sy = nx.sy;
            mz.path_len = nx.path_len;
            mz.spawn1 = nx.spawn1;
            mz.status |= nx.status;
            env.mazes[m] = mz;
        }
    } else {
        generate_one(env, g, m);
    }
    __atomic_thread_fence(__ATOMIC_RELEASE);  // the new rng row before the pending flag
    __syncthreads();
    if (lane == 0) gs_store(st, kGenPending);
}

// mm_env_pregen: every pending maze's next maze, generated from its current
// MT state.  A block (one wavefront) scans 64 mazes' states with one load per
// lane, then generates the pending ones, each claimed with a CAS.  Usually
// only a few mazes per step are pending, so the launch is mostly the scan.
__global__ __launch_bounds__(64) void k_pregen(mm_env_t env) {
    __shared__ GenLds g;
    const int lane = threadIdx.x;
    for (int base = blockIdx.x * 64; base < env.n; base += gridDim.x * 64) {
        const int mine = base + lane;
        const bool pend = mine < env.n && __hip_atomic_load(env.gen_state + mine, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT) == kGenPending;
        uint64_t todo = __ballot(pend);
        while (todo) {
            const int m = base + __ffsll((unsigned long long)todo) - 1;
            todo &= todo - 1;
            if (lane == 0) g.claim = gs_cas(env.gen_state + m, kGenPending, kGenRunning);
            __syncthreads();
            if (g.claim) {
                __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the rng row the reset released
                generate_into(env, g, env.rng + (size_t)m * MM_RNG_WORDS, env.next_rng + (size_t)m * MM_RNG_WORDS,
                              env.next_layout + (size_t)m * env.layout_stride, env.next_mazes + m, true);
                __atomic_thread_fence(__ATOMIC_RELEASE);
                __syncthreads();
                if (lane == 0) gs_store(env.gen_state + m, kGenReady);
            }
            __syncthreads();
        }
    }
}

// Agent resets + the two reset observations (maze.py:64-71), one thread per
// maze, reading the freshly generated layout from global memory.
__device__ void reset_observe(const mm_env_t& env, int m, float* obs, uint8_t* masks) {
    mm_maze_t mz = env.mazes[m];
    View v;
    v.L = env.layout + (size_t)m * env.layout_stride;
    v.w = mz.w; v.h = mz.h; v.ex = mz.ex; v.ey = mz.ey; v.kx = mz.kx; v.ky = mz.ky;
    v.t = 0; v.max_t = env.max_timestep;
    Agent a0 = load_agent(env.agents[2 * m], 2);
    Agent a1 = load_agent(env.agents[2 * m + 1], 3);
    float* o = obs + (size_t)m * 2 * kObs;
    uint8_t* mk = masks + (size_t)m * 2 * kMask;
    // agent 0 resets and observes while agent 1 still holds its previous state (Q3)
    reset_agent(a0, mz.sx, mz.sy);
    observe(v, a0, a1, false, [&](int i, float x) { o[i] = x; }, mk);
    reset_agent(a1, mz.spawn1 & 0xff, (mz.spawn1 >> 8) & 0xff);
    observe(v, a1, a0, true, [&](int i, float x) { o[kObs + i] = x; }, mk + kMask);
    env.agents[2 * m] = pack_agent(a0);
    env.agents[2 * m + 1] = pack_agent(a1);
}

__global__ __launch_bounds__(256) void k_reset_obs(mm_env_t env, const uint8_t* __restrict__ mask, int use_list,
                                                   float* obs, uint8_t* masks) {
    const int count = use_list ? min(env.work[0], env.n) : env.n;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < count; k += gridDim.x * blockDim.x) {
        const int m = use_list ? env.work[kListOff + k] : k;
        if (!use_list && mask && !mask[m]) continue;
        reset_observe(env, m, obs, masks);
    }
    if (use_list) {
        // Done list consumed: the LAST block to finish clears the counter for
        // the next step (every block read work[0] above, before taking its
        // ticket).  Kernel boundaries order this against the next k_step.
        __syncthreads();
        if (threadIdx.x == 0) {
            const int ticket = atomicAdd(&env.work[1], 1);
            if (ticket == (int)gridDim.x - 1) {
                env.work[0] = 0;
                env.work[1] = 0;
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_reset(mm_env_t env, const uint8_t* __restrict__ mask, int use_list,
                                              float* obs, uint8_t* masks) {
    __shared__ GenLds g;
    const int count = use_list ? min(env.work[0], env.n) : env.n;
    for (int k = blockIdx.x; k < count; k += gridDim.x) {
        const int m = use_list ? env.work[kListOff + k] : k;
        if (!use_list && mask && !mask[m]) continue;
        reset_one(env, g, m);
        __syncthreads();
    }
}

// The done-list reset of the rollout (mm_env_step's auto-reset, mm_env_reset_done) in ONE launch: workgroup b
// (one wavefront) regenerates its list entries b, b + G, ... one after another (k_reset's work), then its lanes
// form their reset observations in parallel, lane j for its j-th maze (k_reset_obs's work), after a barrier
// that orders the new layouts / maze records before the reads; the last workgroup clears the list.  Per step
// at a few thousand mazes the two launches were two latency floors (~5 us each plus the gap between them).
__global__ __launch_bounds__(64) void k_reset_list(mm_env_t env, float* obs, uint8_t* masks) {
    __shared__ GenLds g;
    const int count = min(env.work[0], env.n);
    const int G = gridDim.x, per = (count + G - 1) / G;  // list entries per workgroup (round-robin)
    for (int j0 = 0; j0 < per; j0 += 64) {
        const int jn = min(64, per - j0);
        for (int j = j0; j < j0 + jn; j++) {
            const int k = blockIdx.x + G * j;  // workgroup-uniform
            if (k < count) {
                reset_one(env, g, env.work[kListOff + k]);
                __syncthreads();
            }
        }
        __syncthreads();  // the wavefront's layout / maze-record writes before the lanes observe them
        const int k = blockIdx.x + G * (j0 + (int)threadIdx.x);
        if ((int)threadIdx.x < jn && k < count) reset_observe(env, env.work[kListOff + k], obs, masks);
        __syncthreads();
    }
    // done list consumed: the LAST block to finish clears the counter (every block read work[0] above, before
    // taking its ticket); kernel boundaries order this against the next k_step
    __syncthreads();
    if (threadIdx.x == 0) {
        const int ticket = atomicAdd(&env.work[1], 1);
        if (ticket == (int)gridDim.x - 1) {
            env.work[0] = 0;
            env.work[1] = 0;
        }
    }
}

// ---------------------------------------------------------------------------
// step (one thread per maze)
// ---------------------------------------------------------------------------
// Four lanes per maze, two in each of the workgroup's two wavefronts: the
// lane of agent a in wavefront h works on agent a's relative directions 2h
// and 2h+1 and writes half h of agent a's observation row.  The moves and
// the reward are computed redundantly by all four lanes; the eight direction
// summaries and the two chained replays' results are exchanged through LDS.
constexpr int kStepThreads = 128;  // two wavefronts
// mazes per workgroup: 32 (two lanes of each wavefront per maze), or 16 for
// layouts over 1 KB (the upper half of each wavefront idles; the workgroup's
// LDS halves, so twice as many workgroups share a CU)
constexpr int kMPBig = 16, kMPBigStride = 1024;

// LDS of k_step: the workgroup's layouts, later overlaid by its staged obs and
// mask rows, then the direction summaries (8 words per maze)
template <int MPB>
__host__ __device__ inline int step_sum_off(int stride) {
    const int lay = MPB * stride, rows = MPB * 2 * (kObs * 4 + kMask);
    return ((lay > rows ? lay : rows) + 15) & ~15;
}
template <int MPB>
constexpr int xchg_bytes() { return MPB * 2 * 64; }  // two replay records per maze
// replay records: in the gap between the layouts and the end of the obs
// staging area when it is large enough (10x10 mazes: 5.4 KB), else after the
// summaries -- either way they are dead before the rows are staged
template <int MPB>
__host__ __device__ inline int step_xchg_off(int stride) {
    const int lay = (MPB * stride + 15) & ~15, rows = MPB * 2 * (kObs * 4 + kMask);
    return lay + xchg_bytes<MPB>() <= rows ? lay : step_sum_off<MPB>(stride) + MPB * 8 * 4;
}

// Replay hand-off record (4 x int4): the replayed agent's fields that
// replay() changes, the other agent's flags, and the ray visibility masks.
__device__ __forceinline__ void put_replay(int4* r, const Agent& s, int qflags, const Vis& vis) {
    r[0] = make_int4(s.flags, s.tfls, s.olsx, s.olsy);
    r[1] = make_int4(s.exit_len, s.minx, s.maxx, s.miny);
    r[2] = make_int4(s.maxy, qflags, vis.va, vis.vk);
    r[3] = make_int4(vis.vad, 0, 0, 0);
}

__device__ __forceinline__ void get_replay(const int4* r, Agent& s, int& qflags, Vis& vis) {
    const int4 w0 = r[0], w1 = r[1], w2 = r[2], w3 = r[3];
    s.flags = w0.x; s.tfls = w0.y; s.olsx = w0.z; s.olsy = w0.w;
    s.exit_len = w1.x; s.minx = w1.y; s.maxx = w1.z; s.miny = w1.w;
    s.maxy = w2.x; qflags = w2.y; vis.va = w2.z; vis.vk = w2.w;
    vis.vad = w3.x;
}

// LAT (latency form, chosen when the grid is at most two workgroups per CU: one round, one wavefront per
// SIMD, so the launch is the per-maze critical chain): every lane replays both agents itself, in the
// reference's order, instead of handing the two replays between the wavefronts (two barriers and two LDS
// records); and in the 16-maze workgroups of layouts over 1 KB the otherwise idle upper half of each
// wavefront takes one of the lane's two relative directions, so each lane summarises one ray, not two
template <int MPB, bool LAT>
__global__ __launch_bounds__(kStepThreads) void k_step(mm_env_t env, const int8_t* __restrict__ act,
                                                        float* __restrict__ obs, uint8_t* __restrict__ masks,
                                                        float* __restrict__ reward, uint8_t* __restrict__ done,
                                                        int32_t* __restrict__ ep_stats, int list_done) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int stride = env.layout_stride;
    const int m0 = blockIdx.x * MPB;
    const int nb = min(MPB, env.n - m0);
    // wavefront h (0, 1) works on relative directions 2h, 2h+1 of both agents
    // and builds half h of their observation rows; lane l of a wavefront:
    // maze l >> 1, agent l & 1.  h is wavefront-uniform, so each wavefront
    // computes only its half of the observation.
    const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr bool kDSplit = LAT && MPB == kMPBig;  // upper half-wavefront: the lane's second direction
    const int lm = kDSplit ? (threadIdx.x & 31) >> 1 : (threadIdx.x & 63) >> 1;  // maze within the workgroup
    const int dsl = kDSplit ? (threadIdx.x >> 5) & 1 : 0;
    const int a = threadIdx.x & 1;
    const bool lead = h == 0 && a == 0 && dsl == 0;  // writes the maze's marks and state to HBM
    const int m = m0 + lm;
    const bool valid0 = lm < nb;     // moves and direction summaries (both half-wavefronts when kDSplit)
    const bool valid = valid0 && dsl == 0;
#ifdef MM_STEP_STAMPS  // tools/step_stamps.py: per-workgroup phase clocks into work[64 + 12*block]
    uint64_t st[10];
    st[0] = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#define MM_STAMP(i) st[i] = __builtin_amdgcn_s_memtime()
#else
#define MM_STAMP(i)
#endif
    // the layout DMA is issued first, then the per-maze state loads; all of
    // them are in flight together until the staging barrier
    copy_in(smem, env.layout + (size_t)m0 * stride, nb * stride);
    mm_maze_t mz{};
    mm_agent_t g0{}, g1{};
    char4 ac{};
    if (valid0) {
        mz = env.mazes[m];
        g0 = env.agents[2 * m];
        g1 = env.agents[2 * m + 1];
        ac = reinterpret_cast<const char4*>(act)[m];
    }
    __syncthreads();
    MM_STAMP(1);
    View v;
    v.L = smem + lm * stride;
    v.w = mz.w; v.h = mz.h; v.ex = mz.ex; v.ey = mz.ey; v.kx = mz.kx; v.ky = mz.ky;
    v.max_t = env.max_timestep;
    Agent a0 = load_agent(g0, 2);
    Agent a1 = load_agent(g1, 3);
    uint32_t status = mz.status;
    int first_key = 0, have_key = 0;
    if (valid0) {
        // maze.py:75-90: both wavefronts replay the moves and write the same
        // mark bytes into LDS; the lead lane also writes them to HBM
        uint8_t* gl = lead ? env.layout + (size_t)m * stride : nullptr;
        mz.t += 1;
        v.t = mz.t;
        first_key = agent_step(v, a0, ac.x, ac.y, gl, status);
        const int have_key0 = a0.f(MM_AF_HAS_KEY);
        first_key += agent_step(v, a1, ac.z, ac.w, gl, status);
        have_key = have_key0 + a1.f(MM_AF_HAS_KEY);
    }
    // the other wavefront's writes of the same mark bytes (possibly
    // interleaved with ours) are done before any ray reads the marks
    __syncthreads();
    MM_STAMP(5);
    // direction summaries of the maze, [agent][relative direction]
    uint32_t* ssum = reinterpret_cast<uint32_t*>(smem + step_sum_off<MPB>(stride)) + 8 * lm;
    if (valid0) {  // geometry of this lane's two directions of agent a (kDSplit: its one direction)
        const Agent me0 = a ? a1 : a0, ot0 = a ? a0 : a1;
        if constexpr (kDSplit) {
            ssum[4 * a + 2 * h + dsl] =
                summarize_dir(v, me0.x, me0.y, me0.dir, 2 * h + dsl, me0.tag, ot0.x, ot0.y, true);
        } else {
            const uint32_t sA = summarize_dir(v, me0.x, me0.y, me0.dir, 2 * h, me0.tag, ot0.x, ot0.y, true);
            const uint32_t sB = summarize_dir(v, me0.x, me0.y, me0.dir, 2 * h + 1, me0.tag, ot0.x, ot0.y, true);
            *reinterpret_cast<uint2*>(ssum + 4 * a + 2 * h) = make_uint2(sA, sB);
        }
    }
    __syncthreads();
    MM_STAMP(6);
    uint32_t sum0[4], sum1[4];
    if (valid) {
        const uint4 s0 = *reinterpret_cast<const uint4*>(ssum), s1 = *reinterpret_cast<const uint4*>(ssum + 4);
        sum0[0] = s0.x; sum0[1] = s0.y; sum0[2] = s0.z; sum0[3] = s0.w;
        sum1[0] = s1.x; sum1[1] = s1.y; sum1[2] = s1.z; sum1[3] = s1.w;
    }
    // maze.py:99-106: agent 0 observes (may update agent 1), then agent 1.
    // The two replays form a chain: wavefront 0 replays agent 0, wavefront 1
    // then replays agent 1, and each hands its result to the other through
    // LDS (one record per replay and maze), so every replay runs once.
    Vis r0{0, 0, 0}, r1{0, 0, 0};
    Agent a0_obs = a0;  // agent 0's observation is taken after its replay, before agent 1 may update it
    if constexpr (LAT) {  // both replays in every lane, in order (no hand-offs)
        if (valid) {
            r0 = replay(v, a0, a1, sum0);
            a0_obs = a0;
            r1 = replay(v, a1, a0, sum1);
        }
    } else {
        int4* xrec = reinterpret_cast<int4*>(smem + step_xchg_off<MPB>(stride)) + 8 * lm;  // [replay][4 x int4]
        if (valid && h == 0) {
            r0 = replay(v, a0, a1, sum0);
            if (a == 0) put_replay(xrec, a0, a1.flags, r0);
        }
        __syncthreads();
        a0_obs = a0;
        if (valid && h == 1) {
            int f1 = a1.flags;
            get_replay(xrec, a0, f1, r0);
            a1.flags = f1;
            a0_obs = a0;
            r1 = replay(v, a1, a0, sum1);
            if (a == 0) put_replay(xrec + 4, a1, a0.flags, r1);
        }
        __syncthreads();
        if (valid && h == 0) {
            int f0 = a0.flags;
            get_replay(xrec + 4, a1, f0, r1);
            a0.flags = f0;
        }
    }
    const bool exit_ready = a0_obs.f(MM_AF_TEAM_KEY) && a0_obs.f(MM_AF_KNOWS_END) && a1.f(MM_AF_TEAM_KEY) &&
                            a1.f(MM_AF_KNOWS_END);
    MM_STAMP(7);
    float oh[33];  // this wavefront's half of the observation row
    uint8_t mk[kMask];
    if (valid) {
        const Agent me = a ? a1 : a0_obs;
        const Vis rm = a ? r1 : r0;
        uint32_t sm[4];
#pragma unroll
        for (int d = 0; d < 4; d++) sm[d] = a ? sum1[d] : sum0[d];
        float o[kObs];
        if (h == 0) {  // elements [0, 33) and the action mask
            const int am = build_obs(v, me, rm, sm, o, mk);
            if (exit_ready) {  // maze.py:107-113
                if (!v.is_end(me.x, me.y)) {
#pragma unroll
                    for (int d = 0; d < 4; d++) mk[d] = (uint8_t)(d == am);
                } else {
                    mk[0] = mk[1] = mk[2] = mk[3] = 0;
                    mk[4] = 1;
                }
            }
#pragma unroll
            for (int k = 0; k < 33; k++) oh[k] = o[k];
        } else {  // elements [33, 65); the compiler drops the rest of build_obs
            uint8_t unused[kMask];
            build_obs(v, me, rm, sm, o, unused);
#pragma unroll
            for (int k = 0; k < 32; k++) oh[k] = o[33 + k];
            oh[32] = 0.f;
        }
    }
    MM_STAMP(2);
    // The workgroup's obs rows [2*m0, 2*(m0+nb)) and mask rows are contiguous
    // in HBM: stage them in LDS (over the layouts, which are no longer read)
    // and store them with 16-byte coalesced writes.
    __syncthreads();
    float* sobs = reinterpret_cast<float*>(smem);
    uint8_t* smk = smem + MPB * 2 * kObs * 4;
    if (valid) {
        float* orow = sobs + (2 * lm + a) * kObs + 33 * h;  // wavefront h: elements [33h, 33h + 33 - h)
#pragma unroll
        for (int k = 0; k < 33; k++)
            if (k < 32 || h == 0) orow[k] = oh[k];
        if (h == 0) {
#pragma unroll
            for (int i = 0; i < kMask; i++) smk[(2 * lm + a) * kMask + i] = mk[i];
        }
    }
    __syncthreads();
    MM_STAMP(3);
    copy_out(reinterpret_cast<uint8_t*>(obs + (size_t)2 * m0 * kObs), smem, nb * 2 * kObs * 4);
    copy_out(masks + (size_t)2 * m0 * kMask, smk, nb * 2 * kMask);
    MM_STAMP(4);
#ifdef MM_STEP_STAMPS
    if (threadIdx.x == 0) {
        int32_t* w = env.work + kListOff + 12 * blockIdx.x;
        for (int i = 1; i < 5; i++) w[i - 1] = (int32_t)(st[i] - st[0]);
        w[4] = (int32_t)(uint32_t)rt0;
        w[5] = (int32_t)(uint32_t)__builtin_amdgcn_s_memrealtime();
        w[6] = (int32_t)(st[5] - st[0]);
        w[7] = (int32_t)(st[6] - st[5]);  // summaries
        w[8] = (int32_t)(st[7] - st[6]);  // replays
    }
#endif
    if (!valid || !lead) return;
    // reward / done (maze.py:115-121) and state write-back
    float r = first_key ? 0.5f * first_key : 0.f;
    uint8_t dn = 0;
    if (have_key && a0.x == a1.x && a0.y == a1.y && v.is_end(a0.x, a0.y)) {
        r = 1.f;
        dn = 1;
    } else if (mz.t >= env.max_timestep) {
        dn = 1;
    }
    __builtin_nontemporal_store(r, reward + m);
    __builtin_nontemporal_store(dn, done + m);
    if (ep_stats) {  // (episode length, shortest_path_len) of an episode that ended here (PPO.py:129,131)
        const uint64_t es = dn ? ((uint64_t)(uint32_t)mz.path_len << 32) | (uint32_t)mz.t : 0ull;
        __builtin_nontemporal_store(es, reinterpret_cast<uint64_t*>(ep_stats) + m);
    }
    mz.kx = (int8_t)v.kx;
    mz.ky = (int8_t)v.ky;
    mz.status = (uint16_t)status;
    if (dn) {
        mz.episodes += 1;
        mz.last_len = mz.t;
        mz.last_path = mz.path_len;
        if (list_done) {
            const int pos = atomicAdd(&env.work[0], 1);
            if (pos < env.n) env.work[kListOff + pos] = m;  // (queue not drained by the caller: ignore)
        }
    }
    store_nt32(env.mazes + m, mz);
    store_nt32(env.agents + 2 * m, pack_agent(a0));
    store_nt32(env.agents + 2 * m + 1, pack_agent(a1));
}

template <int MPB>
inline size_t step_lds_bytes(int stride) {
    const size_t sums_end = (size_t)step_sum_off<MPB>(stride) + MPB * 8 * 4;
    const size_t xchg_end = (size_t)step_xchg_off<MPB>(stride) + xchg_bytes<MPB>();
    return sums_end > xchg_end ? sums_end : xchg_end;
}

#ifndef STEP_LAT_PER_CU
#define STEP_LAT_PER_CU 2  // layouts up to 1 KB: k_step's latency form for grids of at most this many workgroups
                           // per CU (at 65,536 10x10 mazes both forms measure the same)
#endif

// compute units of the current device (cached per device)
static int cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 256;
    return cus[dev];
}

inline int check_env(const mm_env_t* env) {
    if (!env || env->n <= 0 || !env->layout || !env->agents || !env->mazes || !env->rng || !env->work) return MM_E_ARG;
    const int need = mm_layout_stride(env->size_w, env->size_h, env->rand_sizes, env->rand_lo, env->rand_hi);
    if (need < 0 || env->size_w < 2 || env->size_h < 2) return MM_E_SIZE;
    if (env->rand_sizes && (env->rand_lo < 2 || env->rand_hi < env->rand_lo)) return MM_E_SIZE;
    if (env->layout_stride < need) return MM_E_SIZE;
    // k_step stages the layouts by 16-byte LDS-DMA; the state records are 32-byte structs
    if ((reinterpret_cast<uintptr_t>(env->layout) | reinterpret_cast<uintptr_t>(env->agents) |
         reinterpret_cast<uintptr_t>(env->mazes)) & 15)
        return MM_E_ARG;
    if (env->difficulty < 1 || env->max_timestep < 1) return MM_E_ARG;
    const int npg = !!env->next_layout + !!env->next_mazes + !!env->next_rng + !!env->gen_state;
    if (npg != 0 && npg != 4) return MM_E_ARG;  // the pre-generation buffers come as a set
    if ((reinterpret_cast<uintptr_t>(env->next_layout) | reinterpret_cast<uintptr_t>(env->next_mazes)) & 15)
        return MM_E_ARG;
    return 0;
}

}  // namespace mm

using namespace mm;

extern "C" int mm_version(void) { return 307; }

extern "C" int mm_env_desc_size(void) { return (int)sizeof(mm_env_t); }

extern "C" int mm_layout_stride(int size_w, int size_h, int rand_sizes, int rand_lo, int rand_hi) {
    const int side = rand_sizes ? 2 * rand_hi - 1 : 2 * (size_w > size_h ? size_w : size_h) - 1;
    if (side > MM_MAX_SIDE || side < 3) return MM_E_SIZE;
    const int w = rand_sizes ? side : 2 * size_w - 1, h = rand_sizes ? side : 2 * size_h - 1;
    return w * h;
}

extern "C" int mm_env_seed(const mm_env_t* env, const uint64_t* seeds, void* stream) {
    int e = check_env(env);
    if (e) return e;
    if (!seeds) return MM_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_seed, dim3((env->n + 255) / 256), dim3(256), 0, s, *env, seeds);
    return (int)hipGetLastError();
}

static int launch_reset(const mm_env_t* env, const uint8_t* mask, int use_list, float* obs, uint8_t* masks,
                        hipStream_t s) {
    if (use_list) {
        hipLaunchKernelGGL(k_reset_list, dim3(512), dim3(64), 0, s, *env, obs, masks);
        return (int)hipGetLastError();
    }
    int grid = use_list ? 512 : (env->n < 16384 ? env->n : 16384);
    hipLaunchKernelGGL(k_reset, dim3(grid), dim3(64), 0, s, *env, mask, use_list, obs, masks);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    const int ogrid = use_list ? 256 : (env->n + 255) / 256;
    hipLaunchKernelGGL(k_reset_obs, dim3(ogrid), dim3(256), 0, s, *env, mask, use_list, obs, masks);
    return (int)hipGetLastError();
}

extern "C" int mm_env_reset(const mm_env_t* env, const uint8_t* reset_mask, float* obs, uint8_t* masks, void* stream) {
    int e = check_env(env);
    if (e) return e;
    if (!obs || !masks) return MM_E_ARG;
    return launch_reset(env, reset_mask, 0, obs, masks, (hipStream_t)stream);
}

extern "C" int mm_env_step_timed(const mm_env_t* env, const int8_t* actions, float* obs, uint8_t* masks,
                                 float* reward, uint8_t* done, int32_t* ep_stats, int auto_reset, void* stream,
                                 void* ev_start, void* ev_stop) {
    int e = check_env(env);
    if (e) return e;
    if (!actions || !obs || !masks || !reward || !done) return MM_E_ARG;
    if (auto_reset < 0 || auto_reset > 2) return MM_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    // hipExtLaunchKernel stamps the events at the kernel's own start / end
    if (env->layout_stride > kMPBigStride) {
        // large layouts: the latency form at every size (its split directions put the otherwise idle upper
        // half-wavefronts to work: 65,536 20x20 mazes 38.7-39.9 -> 36.0 us, the same A/B on one box)
        const int grid = (env->n + kMPBig - 1) / kMPBig;
        const size_t lds = step_lds_bytes<kMPBig>(env->layout_stride);
        hipExtLaunchKernelGGL((k_step<kMPBig, true>), dim3(grid), dim3(kStepThreads), (uint32_t)lds, s,
                              (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0, *env, actions, obs, masks, reward, done,
                              ep_stats, auto_reset ? 1 : 0);
    } else {
        const int grid = (env->n + 2 * kMPBig - 1) / (2 * kMPBig);
        const size_t lds = step_lds_bytes<2 * kMPBig>(env->layout_stride);
        if (grid <= STEP_LAT_PER_CU * cu_count())
            hipExtLaunchKernelGGL((k_step<2 * kMPBig, true>), dim3(grid), dim3(kStepThreads), (uint32_t)lds, s,
                                  (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0, *env, actions, obs, masks, reward,
                                  done, ep_stats, auto_reset ? 1 : 0);
        else
            hipExtLaunchKernelGGL((k_step<2 * kMPBig, false>), dim3(grid), dim3(kStepThreads), (uint32_t)lds, s,
                                  (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0, *env, actions, obs, masks, reward,
                                  done, ep_stats, auto_reset ? 1 : 0);
    }
    hipError_t le = hipGetLastError();
    if (le != hipSuccess) return (int)le;
    if (auto_reset == 1) return launch_reset(env, nullptr, 1, obs, masks, s);
    return 0;
}

extern "C" int mm_env_step(const mm_env_t* env, const int8_t* actions, float* obs, uint8_t* masks, float* reward,
                           uint8_t* done, int32_t* ep_stats, int auto_reset, void* stream) {
    return mm_env_step_timed(env, actions, obs, masks, reward, done, ep_stats, auto_reset, stream, nullptr, nullptr);
}

extern "C" int mm_env_pregen(const mm_env_t* env, void* stream) {
    int e = check_env(env);
    if (e) return e;
    if (!env->gen_state) return MM_E_ARG;
    const int chunks = (env->n + 63) / 64;
    const int grid = chunks < 256 ? chunks : 256;  // one block per CU: little LDS held beside the step kernels
    hipLaunchKernelGGL(k_pregen, dim3(grid), dim3(64), 0, (hipStream_t)stream, *env);
    return (int)hipGetLastError();
}

extern "C" int mm_env_reset_done(const mm_env_t* env, float* obs, uint8_t* masks, void* stream) {
    int e = check_env(env);
    if (e) return e;
    if (!obs || !masks) return MM_E_ARG;
    return launch_reset(env, nullptr, 1, obs, masks, (hipStream_t)stream);
}
