/*
 * marlmaze.h -- C ABI of the MI355X (gfx950) MARL-Maze hot path.
 *
 * Library: marl-maze_amd/libmarlmaze.so (hipcc --offload-arch=gfx950).
 *
 * The reference (rhuangr/MARL-Maze) is pure Python and has no FFI; the entry
 * points below are what its Python classes would bind to run the hot path on
 * the GPU.  Each cites the reference interface it replaces:
 *
 *   mm_env_seed   random.seed(s) before Maze.reset()           (maze.py:170-259 draws
 *                                                              from the global `random`)
 *   mm_env_reset  Maze.reset()                                  maze.py:55-72
 *   mm_env_step   Maze.step(action) (+ PPO.get_batch's reset     maze.py:74-163,
 *                 on done, PPO.py:127-130)                      maze_agent.py:89-358
 *   mm_gae        PPO.get_GAEs                                  PPO.py:193-203
 *   mm_sample     PPO.get_action (masked Categorical move +     PPO.py:170-186
 *                 Bernoulli mark, joint log-prob)
 *
 * Conventions
 *   - Every pointer is a caller-owned DEVICE buffer (e.g. a torch tensor);
 *     the library never allocates, frees or synchronises.  All work is
 *     enqueued on `stream` (a hipStream_t passed as void*; NULL = default
 *     stream) and is graph-capturable.
 *   - Return value: 0 on success, otherwise a hipError_t from the launch or a
 *     negative MM_E* code for invalid arguments.  Device-side failures (an
 *     illegal move, a maze whose key cannot be placed: maze.py:254 loops
 *     forever there) set bits in mm_maze_t.status instead.
 *   - Layout bytes: bits 0-1 = the reference's cell value (0 path, 1 wall,
 *     2/3 = mark of the agent with that tag, maze.py:133), bits 2-4 = the
 *     direction of the next step toward the exit (0..3 = N,E,S,W as
 *     maze.py:19 DELTAS; 4 = this is the exit).  The reference's per-agent
 *     exit_route stack (maze.py:148-154) always equals the tree path, so the
 *     table replaces it.
 *   - Observation row = 65 f32 in Appendix-A order (maze_agent.py:89-130);
 *     mask row = 6 bytes (0/1), maze_agent.py:132-139 + maze.py:107-113.
 */
#ifndef MARLMAZE_H
#define MARLMAZE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MM_OBS_DIM 65
#define MM_MASK_DIM 6
#define MM_RNG_WORDS 625   /* CPython random.getstate()[1]: 624 words + index */
#define MM_MAX_SIDE 41     /* layout side limit (default_size <= 21) */
#define MM_MAZES_PER_BLOCK 32  /* mazes per env-step workgroup (4 lanes each); 16 when layout_stride > 1024 */

#define MM_E_ARG (-1)
#define MM_E_SIZE (-2)

/* mm_maze_t.status bits */
#define MM_ST_GEN_FAIL 1u      /* set_key/set_end found no cell (reference hangs) */
#define MM_ST_BAD_MOVE 2u      /* an action moved into a wall / off the grid */

/* Per-agent state: 32 bytes (maze_agent.py:16-79). */
typedef struct {
    int8_t x, y, dir, flags;        /* flags: MM_AF_* */
    int8_t lmx, lmy, olsx, olsy;    /* last_mark_pos, other_last_seen */
    int8_t minx, maxx, miny, maxy;  /* *_visited (Q9) */
    int8_t mem[4];                  /* deque(maxlen=4) of relative moves, -1 = empty */
    int32_t exit_len;               /* maze_agent.py:33 */
    int32_t tfls;                   /* time_from_last_seen, never reset (Q5) */
    int32_t reserved[2];
} mm_agent_t;

#define MM_AF_KNOWS_END 1
#define MM_AF_SEES_END 2
#define MM_AF_OTHER_KNOWS 4
#define MM_AF_HAS_KEY 8
#define MM_AF_SEES_KEY 16
#define MM_AF_TEAM_KEY 32
#define MM_AF_HAS_MARK 64

/* Per-maze scalars: 32 bytes (maze.py:22-53). */
typedef struct {
    int32_t t;            /* current_t */
    int8_t w, h;          /* width, height (2*size-1) */
    int8_t ex, ey;        /* end */
    int8_t kx, ky;        /* key; kx = -1 after pickup (maze.py:157-158) */
    int8_t sx, sy;        /* start */
    int16_t path_len;     /* shortest_path_len */
    uint16_t status;      /* MM_ST_* */
    int32_t episodes;     /* completed episodes */
    int32_t last_len;     /* length of the last completed episode */
    int32_t last_path;    /* shortest_path_len of the last completed episode */
    int32_t spawn1;       /* shortest_path[1] = agent 1's spawn, x | y << 8 (maze.py:66) */
} mm_maze_t;

/* Environment descriptor (host struct holding device pointers). */
typedef struct {
    int32_t n;                     /* number of mazes */
    int32_t size_w, size_h;        /* default_size in cells (maze.py:23) */
    int32_t max_timestep;          /* maze.py:22 */
    int32_t difficulty;            /* maze.py:22 */
    int32_t rand_start;            /* maze.py:22 */
    int32_t rand_sizes;            /* maze.py:23 */
    int32_t rand_lo, rand_hi;      /* rand_range */
    int32_t layout_stride;         /* bytes per maze layout (>= side_max^2) */
    uint8_t* layout;               /* [n, layout_stride], 16-byte aligned (as agents, mazes) */
    mm_agent_t* agents;            /* [n, 2] */
    mm_maze_t* mazes;              /* [n] */
    uint32_t* rng;                 /* [n, MM_RNG_WORDS] */
    int32_t* work;                 /* [n + 64] scratch (done list) */
    /* Optional pre-generation (all four NULL: every reset generates inline).
     * Maze generation depends only on the maze's own MT19937 stream
     * (maze.py:170-259), so each maze's NEXT maze can be generated ahead, off
     * the step's critical path, by mm_env_pregen on a side stream; a reset
     * then copies it in.  gen_state[i]: 0 = next_* hold the next maze,
     * 1 = pending (mm_env_pregen will generate it), 2 = mm_env_pregen is
     * generating it, 3 = a reset is generating inline.  rng always holds the
     * state after the CURRENT maze's generation (the reference's observable
     * random state), next_rng the state after the next one. */
    uint8_t* next_layout;          /* [n, layout_stride], 16-byte aligned */
    mm_maze_t* next_mazes;         /* [n]: generation fields of the next maze */
    uint32_t* next_rng;            /* [n, MM_RNG_WORDS] */
    int32_t* gen_state;            /* [n] */
} mm_env_t;

/* Library version (major*100 + minor).  The major number changes whenever a
 * struct of this header changes (3: mm_env_t has its 19 fields). */
int mm_version(void);

/* sizeof(mm_env_t) as compiled into the library: a binding that mirrors the
 * struct (ctypes, cffi, cgo) compares its own size with this before the first
 * call -- mm_env_t is passed by pointer, so a short mirror would otherwise make
 * the library read past the caller's struct. */
int mm_env_desc_size(void);

/* Bytes needed for layout_stride given the config (side_max^2). */
int mm_layout_stride(int size_w, int size_h, int rand_sizes, int rand_lo, int rand_hi);

/* random.seed(seeds[i]) for every maze i; also initialises the agents as
 * Agent.__init__ does (x=y=0, facing south; maze_agent.py:24-57).
 * seeds: device [n] uint64. */
int mm_env_seed(const mm_env_t* env, const uint64_t* seeds, void* stream);

/* Maze.reset() for the mazes with reset_mask[i] != 0 (reset_mask may be NULL
 * = all).  Writes obs [n,2,65] f32 and masks [n,2,6] u8 rows of those mazes. */
int mm_env_reset(const mm_env_t* env, const uint8_t* reset_mask, float* obs, uint8_t* masks, void* stream);

/* Maze.step(actions) for every maze.  actions [n,2,2] int8 = (move, mark) per
 * agent.  Outputs obs [n,2,65] f32, masks [n,2,6] u8, reward [n] f32,
 * done [n] u8, and (if ep_stats != NULL) ep_stats [n,2] int32 = (episode
 * length, shortest_path_len) where done, (0,0) elsewhere (PPO.py:129,131).
 * auto_reset = 1: the finished mazes are regenerated and their obs/mask rows
 * replaced by the reset observation (PPO.py:127-130); = 2: the finished
 * mazes are only queued, for a later mm_env_reset_done (lets a caller time
 * or overlap the step kernel alone); = 0: nothing is reset or queued. */
int mm_env_step(const mm_env_t* env, const int8_t* actions, float* obs, uint8_t* masks, float* reward, uint8_t* done,
                int32_t* ep_stats, int auto_reset, void* stream);

/* mm_env_step whose step kernel is launched with hipExtLaunchKernel: the two
 * hipEvent_t (created by the caller with timing enabled; either may be NULL)
 * are stamped at the step kernel's own start and end, so their elapsed time is
 * the kernel's duration (used by bench.py for the roofline). */
int mm_env_step_timed(const mm_env_t* env, const int8_t* actions, float* obs, uint8_t* masks, float* reward,
                      uint8_t* done, int32_t* ep_stats, int auto_reset, void* stream, void* ev_start, void* ev_stop);

/* Maze.reset() for the mazes queued by the previous mm_env_step(auto_reset=2)
 * (writes their obs/mask rows; clears the queue). */
int mm_env_reset_done(const mm_env_t* env, float* obs, uint8_t* masks, void* stream);

/* Generate the next maze of every maze whose gen_state is 1 (pending) into
 * next_layout / next_mazes / next_rng (needs the pre-generation buffers).
 * Safe to run on a second stream concurrently with steps and resets of the
 * same env: mazes are claimed with atomics, and a reset that finds its maze's
 * next maze still being generated waits for it.  Replaces nothing in the
 * reference (its build_maze runs inside Maze.reset, maze.py:55-72). */
int mm_env_pregen(const mm_env_t* env, void* stream);

/* Time-major GAE over [T, N] (PPO.py:193-203, episodes concatenated in time,
 * done[t] = the transition at t ended its episode).  last_value [N] (may be
 * NULL): bootstrap for segments that end mid-episode; NULL makes every
 * segment end an episode end (done[T-1] := 1: the reference's GAE applied
 * to each episode fragment, PPO.py:197-198).
 * gamma, gamma_lambda are the f32 factors (f32(0.99), f32(0.99*0.95)).
 * adv, rtg = adv + value: [T, N] f32.  Arithmetic is fp32 with no FMA, in
 * the reference's operation order: bit-exact. */
int mm_gae(const float* reward, const float* value, const uint8_t* done, const float* last_value, int T, int N,
           float gamma, float gamma_lambda, float* adv, float* rtg, void* stream);

/* mm_gae with the algorithm chosen by the caller (mm_gae = MM_GAE_AUTO):
 *   MM_GAE_COLUMN  one lane per column, reverse recursion (many columns);
 *   MM_GAE_WALK    one lane per (column, chunk of t) running the episodes that
 *                  end in its chunk (few columns, long T: the reference's
 *                  whole-episode batches, PPO.py:108-141) -- bit-identical to
 *                  MM_GAE_COLUMN, parallel across episodes;
 *   MM_GAE_SCAN    one workgroup per column, affine-map suffix scan with
 *                  wavefront shuffles -- parallel inside an episode,
 *                  reassociated fp32 (not bit-exact; ~1e-7 relative);
 *   MM_GAE_AUTO    COLUMN for N >= 256 or short T, else WALK (bit-exact). */
#define MM_GAE_AUTO 0
#define MM_GAE_COLUMN 1
#define MM_GAE_WALK 2
#define MM_GAE_SCAN 3
int mm_gae_ex(const float* reward, const float* value, const uint8_t* done, const float* last_value, int T, int N,
              float gamma, float gamma_lambda, float* adv, float* rtg, int algo, void* stream);

/* Sample one action per agent row (PPO.py:170-186): move ~ Categorical over
 * move_logits [M,5] masked to -inf where masks[:,0:5]==0; mark ~ Bernoulli(
 * sigmoid(mark_logit [M])) where masks[:,5] else 0.  Rows are (maze, agent)
 * pairs: M = 2N.  actions [M,2] int8; logp [M] per-agent log-prob; joint_logp
 * [N] = logp[2i] + logp[2i+1] (may be NULL).  Counter-based Philox4x32-10
 * keyed by (seed), counter = (offset, row): reproducible and replayable. */
int mm_sample(const float* move_logits, const float* mark_logits, const uint8_t* masks, int M, uint64_t seed,
              uint64_t offset, int8_t* actions, float* logp, float* joint_logp, void* stream);


/* "TP" operands for the pre-split x3 GEMMs (csrc/x3mlp.hip): a logical [R, C]
 * fp32 matrix stored as three exact bf16 planes (x = hi + mid + lo) in MFMA
 * fragment order -- block (rt, ks) of rows 16rt..+15 and columns 32ks..+31 is
 * 3 x 1 KiB [plane][chunk 4][row 16][8 bf16]; R padded to 256, C to 32, pads
 * zero.  mm_x3_tp_len: uint16 elements of such a buffer.
 * mm_x3_tp_pack: fp32 X (row-major with leading dimension ld; trans != 0 reads
 * element (i, j) at X[j * ld + i]) -> TP.  Replaces nothing in the reference:
 * the packed form of nn.Linear operands (networks.py:24-36). */
long mm_x3_tp_len(int R, int C);
int mm_x3_tp_pack(const float* X, int R, int C, int ld, int trans, uint16_t* tp, void* stream);

/* C = A . B^T (+ bias[N]) (ReLU if relu) (* (mask > 0) if mask), B = TP of
 * [N, K]: the nn.Linear forward (B = weight) and input gradient (A = dY, B =
 * TP of weight^T) of networks.py:24-36 / :94-101, with the ReLU-backward of the
 * layer below fused (mask = that layer's output y [M, ldm]: dX *= (y > 0)).
 * mm_x3_nt: A = TP of [M, K].  mm_x3_nt_f32a: A fp32 row-major [M, lda]
 * (K % 4 == 0, lda % 4 == 0, 16-byte aligned), split into bf16 planes inside
 * the GEMM.  Writes fp32 c [M, ldc] and/or the TP c_tp of [M, N] (N <= 272).
 * Accuracy: fp32-class (six bf16 MFMA products per fp32 product). */
int mm_x3_nt(const uint16_t* a_tp, const uint16_t* b_tp, int M, int N, int K, const float* bias, int relu,
             const float* mask, int ldm, float* c, int ldc, uint16_t* c_tp, void* stream);
int mm_x3_nt_f32a(const float* a, int lda, const uint16_t* b_tp, int M, int N, int K, const float* bias, int relu,
                  const float* mask, int ldm, const uint32_t* mbits_in, uint32_t* mbits_out, float* colsum, float* c,
                  int ldc, uint16_t* c_tp, void* stream);
/* ReLU masks as bits in the GEMM's accumulator order (N <= 272, fp32 output):
 * mbits_out (from a forward GEMM with relu) records out > 0; mbits_in (to the
 * next layer's input-gradient GEMM, same [M, N]) multiplies the output by those
 * bits -- the ReLU backward (threshold_backward) without re-reading the
 * activations.  mm_x3_mbits_len: uint32 elements of such a mask for M rows. */
long mm_x3_mbits_len(int M);
/* colsum (with mbits_in): per 16-row tile column sums of the output, [ceil(M / 16), N]
 * -- the next layer down's bias gradient is their column sum (fixed order).
 * mm_x3_heads_bwd: the actor heads' backward (networks.py:38-41) through the
 * last ReLU: dY = (dz [M, J] . W [J, N]) * bits (the last forward GEMM's
 * mbits_out), J <= 8, N <= 272, plus its colsum. */
int mm_x3_heads_bwd(const float* dz, int J, const float* W, const uint32_t* bits, int M, int N, float* dy,
                    float* colsum, void* stream);

/* Precision-generic forms of the actor/critic GEMMs (csrc/x3mlp.hip).
 * prec MM_PREC_X3: bf16x3 operands (six products, fp32-class, as mm_x3_*);
 * MM_PREC_F16: one fp16 plane per operand, one f16 MFMA per product, fp32
 * accumulation (the fp16 actor/critic of BASELINE configs[4]; storage,
 * master weights and optimizer stay fp32).  ascale / dscale multiply the A
 * (dY) operand before its fp16 rounding and cscale the result (powers of two:
 * exact; a gradient far below 1 keeps fp16 precision).  X3 requires 1.0 for
 * all scales.
 * MM_PREC_X2: fp32-class on two fp16 planes per operand: (x s) = hi + 2^-11 lo,
 * hi = RN16(x s), lo = RN16(2^11 (x s - hi)) -- 22 significand bits for
 * 2^-14 <= |x s| <= 2^15 (the 2^11 keeps lo out of the fp16 subnormals), three
 * f16 MFMAs per product (hi hi into one accumulator; hi lo + lo hi into a
 * second, added with weight 2^-11 before the epilogue) instead of X3's six
 * bf16 ones, and two B planes instead of three.  Scales as for F16.
 * mm_gemm_tp_len / mm_gemm_tp_pack: the TP form of B for that precision (P_F16:
 * one 1-KiB plane per block; P_X2: two).
 * mm_gemm_nt: c = cscale (ascale A . B^T) (+ bias)(ReLU) -- mm_x3_nt_f32a's
 * forward (mbits_out) and input-gradient (mbits_in, colsum) forms; A fp32
 * [M, lda] with K, lda % 4 == 0 and 16-byte alignment, or (outputs N <= 64,
 * e.g. the critic's [M, 130] observations) K, lda even and 8-byte alignment.
 * mm_gemm_wgrad: the weight gradient of nn.Linear under autograd (networks.py
 * :35-41, :87-106), dw [N, K] = cscale * sum_m (dscale dy[m, n]) x[m, k], dy
 * [M, lddy], x [M, ldx], N <= 272; row slices' partials in ws
 * [mm_gemm_wgrad_ws_len(M, N, K)] floats, summed in a fixed order. */
#define MM_PREC_X3 0
#define MM_PREC_F16 1
#define MM_PREC_X2 2
long mm_gemm_tp_len(int prec, int R, int C);
int mm_gemm_tp_pack(int prec, const float* X, int R, int C, int ld, int trans, uint16_t* tp, void* stream);
int mm_gemm_nt(int prec, const float* a, int lda, float ascale, const uint16_t* b_tp, int M, int N, int K,
               const float* bias, int relu, const uint32_t* mbits_in, uint32_t* mbits_out, float* colsum, float cscale,
               float* c, int ldc, void* stream);
/* mm_gemm_nt_algo: which kernel mm_gemm_nt / mm_x3_nt_f32a use (process-wide; returns the previous
 * setting).  MM_GEMM_AUTO: the B-resident kernel (a column block of B kept in LDS for the whole launch,
 * independent waves) where the shape fits it (M >= 16384, B block of >= 4 tiles), else the streaming
 * kernel; MM_GEMM_STREAM: always the streaming kernel (B through LDS one k-step at a time).  Initial
 * value: MM_GEMM_STREAM if the environment sets MARLMAZE_GEMM_BRES=0, else MM_GEMM_AUTO. */
#define MM_GEMM_AUTO 0
#define MM_GEMM_STREAM 1
int mm_gemm_nt_algo(int algo);
long mm_gemm_wgrad_ws_len(int M, int N, int K);
/* mm_gemm_wgrad_algo: which kernel the MM_PREC_X2 weight gradients of the actor trunk's shapes (264 x 264,
 * 264 x 460) use (process-wide; returns the previous setting).  MM_WGRAD_DMA: raw rows staged HBM -> LDS by
 * LDS-DMA into a two-stage ring (two steps in flight); MM_WGRAD_REG: staged through registers one step ahead.
 * Bit-identical results.  Initial value: MM_WGRAD_REG if the environment sets MARLMAZE_WG_DMA=0, else
 * MM_WGRAD_DMA.  Replaces nothing in the reference (a kernel choice of networks.py:35-41's backward). */
#define MM_WGRAD_DMA 0
#define MM_WGRAD_REG 1
int mm_gemm_wgrad_algo(int algo);
int mm_gemm_wgrad(int prec, const float* dy, int lddy, float dscale, const float* x, int ldx, int M, int N, int K,
                  float cscale, float* ws, float* dw, void* stream);
/* The update's batched forms (one launch for what a backward would otherwise
 * issue per layer; each result bit-identical to the single form):
 * mm_gemm_tp_pack_multi: nseg <= 16 packs of one precision (mm_gemm_tp_pack's
 * arguments per segment).
 * mm_gemm_wgrad_partials: mm_gemm_wgrad without its final reduction: ws receives
 * mm_gemm_wgrad_slices(prec, M, N, K) row-slice partials of [N, K], summed later
 * by mm_wsum_multi with S = that count (M > 0). */
typedef struct {
    const float* X;
    int R, C, ld, trans;
    uint16_t* tp;
} mm_pack_seg_t;
int mm_gemm_tp_pack_multi(int prec, const mm_pack_seg_t* segs, int nseg, void* stream);
int mm_gemm_wgrad_slices(int prec, int M, int N, int K);
int mm_gemm_wgrad_partials(int prec, const float* dy, int lddy, float dscale, const float* x, int ldx, int M, int N,
                           int K, float cscale, float* ws, void* stream);
/* Range guard of MM_PREC_X2 / MM_PREC_F16 (fp16 planes: |x s| >= 65520 would
 * round to inf, where the fp32 reference stays finite).  The GEMM and
 * weight-gradient kernels of those precisions (mm_gemm_nt(_h),
 * mm_gemm_wgrad(_h, _partials, _partials_h)) OR bit 0 into a library-wide flag
 * when an output accumulator is not finite -- an operand that left fp16's
 * range always makes one -- or, for fp16 outputs (MM_GEMM_C_F16), when a
 * stored value overflowed fp16; the result is then not to be used: redo the
 * work at MM_PREC_X3 (fp32's range).
 * mm_gemm_range_flag: stream-ordered; writes the flag to out[0] (device
 * memory, may be NULL) and, when clear != 0, resets it. */
int mm_gemm_range_flag(uint32_t* out, int clear, void* stream);

/* fp16 activation storage of the MM_PREC_F16 networks (BASELINE configs[4]):
 * the next GEMM rounds every activation to fp16 anyway, so storing them at that
 * precision gives the same operands at half the bytes.  Replaces nothing in
 * the reference (its networks are fp32, networks.py:31-41); used by the
 * update's f16 forward / backward only.
 * The input gradients likewise: stored fp16 as fp16(dY s) -- s the power-of-two
 * scale their consumers apply anyway -- and read back with ascale / dscale 1.
 * mm_gemm_nt_h: mm_gemm_nt with flags -- MM_GEMM_A_F16: a is fp16 [M, lda]
 *   (MM_PREC_F16, ascale 1, K and lda multiples of 4; the B-resident kernel:
 *   mm_gemm_a16_ok says whether the shape takes it); MM_GEMM_C_F16: c is fp16
 *   [M, ldc]: the forward with mbits_out, or the input gradient with mbits_in,
 *   stored as fp16(out * oscale) (its column sums stay those of the fp32 out).
 * mm_gemm_wgrad_h / mm_gemm_wgrad_partials_h: with MM_GEMM_B_F16, x is fp16
 *   [M, ldx] (MM_PREC_F16 at the update's shapes; MM_PREC_X3 for N <= 16,
 *   K <= 272: the actor heads); with MM_GEMM_A_F16, dy is fp16 [M, lddy]
 *   (MM_PREC_F16; dscale 1 for a pre-scaled dY, cscale its inverse scale).
 * mm_x3_heads_bwd_h16: mm_x3_heads_bwd writing dy fp16 = fp16(dY * oscale).
 * mm_heads_fwd_h16: mm_heads_fwd over fp16 h (K 257..288). */
#define MM_GEMM_A_F16 1
#define MM_GEMM_C_F16 2
#define MM_GEMM_B_F16 4
int mm_gemm_nt_h(int prec, int flags, const void* a, int lda, float ascale, const uint16_t* b_tp, int M, int N, int K,
                 const float* bias, int relu, const uint32_t* mbits_in, uint32_t* mbits_out, float* colsum,
                 float cscale, float oscale, void* c, int ldc, void* stream);
int mm_x3_heads_bwd_h16(const float* dz, int J, const float* W, const uint32_t* bits, int M, int N, void* dy,
                        float* colsum, float oscale, void* stream);
int mm_gemm_a16_ok(int M, int N, int K, int lda, int ldc);
int mm_gemm_wgrad_h(int prec, int flags, const float* dy, int lddy, float dscale, const void* x, int ldx, int M, int N,
                    int K, float cscale, float* ws, float* dw, void* stream);
int mm_gemm_wgrad_partials_h(int prec, int flags, const float* dy, int lddy, float dscale, const void* x, int ldx,
                             int M, int N, int K, float cscale, float* ws, void* stream);
int mm_heads_fwd_h16(const void* h, int ldh, int K, const float* w, const float* b, int M, float* logits,
                     void* stream);
/* mm_actor_front_fwd with h stored fp16 [B, 460] (round to nearest of the fp32
 * values): the f16 networks' update, whose first GEMM (fp16 A at K = 460: the
 * streaming kernel) and its weight gradient round h to fp16 anyway. */
int mm_actor_front_fwd_h16(const float* ws, const float* x, int ldx, int B, int parity, void* h, void* stream);
/* mm_actor_front_fwd_h16 with the kernel chosen by `algo` (MM_FRONT_FWD_ROW1 or
 * MM_FRONT_FWD_MFMA, defined below): h16 is the round to nearest of that
 * kernel's fp32 h. */
int mm_actor_front_fwd_h16_ex(const float* ws, const float* x, int ldx, int B, int parity, void* h, int algo,
                              void* stream);

/* The actor trunk's three ReLU layers (networks.py:35-36) in one launch, for
 * the rollout's small row counts (BASELINE configs[1]: 8,192 rows per step,
 * where each layer alone sits at its launch floor).  Replaces three mm_gemm_nt
 * calls (bias, ReLU, no bits); the result is bit-identical to them.
 * out [M, ldc] = relu(relu(relu(h0 W0^T + b0) W1^T + b1) W2^T + b2): h0 fp32
 * [M, lda] (K0 and lda multiples of 4, 16-byte aligned, K0 <= 512), w_l TP
 * packs of [N_l, K_l] in precision prec (K_1 = N0, K_2 = N1), N_l <= 272,
 * b_l [N_l] or NULL.  mm_trunk3_ok: whether the shape is supported (1 / 0). */
int mm_trunk3_ok(int prec, int M, int K0, int N0, int N1, int N2, int lda);
int mm_trunk3(int prec, const float* h0, int lda, int M, int K0, const uint16_t* w0, const float* b0, int N0,
              const uint16_t* w1, const float* b1, int N1, const uint16_t* w2, const float* b2, int N2, float* out,
              int ldc, void* stream);
/* mm_trunk3 + the actor heads + PPO.get_action (PPO.py:170-186) in one launch:
 * the rollout's whole per-step actor after the front-end.  Replaces mm_trunk3
 * followed by mm_head_sample_ex on its output, with the same results bit for
 * bit (head_w [6, N2], head_b [6], masks, seed, offset, offset_dev, actions,
 * logp, joint_logp, logits as there); h3 (optional, [M, ldh3]) receives the
 * trunk's output.  N2 % 4 == 0.  mm_trunk3_head_sample_ok: 1 / 0. */
int mm_trunk3_head_sample_ok(int prec, int M, int K0, int N0, int N1, int N2, int lda);
int mm_trunk3_head_sample(int prec, const float* h0, int lda, int M, int K0, const uint16_t* w0, const float* b0,
                          int N0, const uint16_t* w1, const float* b1, int N1, const uint16_t* w2, const float* b2,
                          int N2, const float* head_w, const float* head_b, const uint8_t* masks, uint64_t seed,
                          uint64_t offset, const uint64_t* offset_dev, int8_t* actions, float* logp,
                          float* joint_logp, float* logits, float* h3, int ldh3, void* stream);

/* The update's policy loss (PPO.py:62-72, get_log_probs PPO.py:154-168),
 * fused: heads [2M, 6] f32 (per agent row: 5 move logits, 1 mark logit),
 * masks [2M, 6] u8, actions [2M, 2] i8 (move, mark); per sample the joint
 * log-prob (sum over the two agents of the masked log-softmax of the move and
 * the masked Bernoulli log-prob of the mark), ratio = exp(logp - old_logp),
 * term = min(ratio A, clamp(ratio, 1 - clip, 1 + clip) A).
 * mm_ppo_loss: partial [mm_ppo_loss_partials(M)] per-workgroup sums of term
 * (the loss is -sum(partial) / M) and coef [M] = d loss / d logp.
 * mm_ppo_loss_bwd: dheads [2M, 6] = dloss[0] * coef * d logp / d heads. */
int mm_ppo_loss_partials(int M);
int mm_ppo_loss(const float* heads, const uint8_t* masks, const int8_t* actions, const float* old_logp,
                const float* adv, int M, float clip, float* coef, float* partial, void* stream);
int mm_ppo_loss_bwd(const float* heads, const uint8_t* masks, const int8_t* actions, const float* coef,
                    const float* dloss, int M, float* dheads, void* stream);

/* The rest of one update minibatch step (PPO.py:58-85; csrc/update_kernels.hip),
 * so that the step is hand-written launches only.  Sums run in a fixed order.
 *
 * mm_colsum: out [N] = column sums of x [R, N] f32 -- the nn.Linear bias
 * gradients (networks.py:35-41, 87-106 under autograd) from the GEMM engine's
 * per-16-row-tile column sums.  Two passes: G slabs of rows into part [G, N]
 * (caller-owned, G >= 1; NULL allowed when G == 1), then the G partials.
 * mm_mse_loss: nn.MSELoss()(V, rtg) (PPO.py:78-80) for V, rtg [M] f32: partial
 * [mm_mse_loss_partials(M)] per-workgroup sums of (V - rtg)^2 and (dv may be
 * NULL) dv [M] = (V - rtg) * (2 / M), the loss's gradient.
 * mm_losses_final: out[0] = -sum(ppo_partial) / M (the actor loss of
 * mm_ppo_loss), out[1] = sum(mse_partial) / M (the critic loss). */
int mm_colsum(const float* x, long R, int N, float* part, int G, float* out, void* stream);
/* mm_colsum_multi: nseg <= 16 column sums in two launches, segment k as
 * mm_colsum(x, R, N, part, min(256, max(1, R / 8)), out) (bit-identical); ws:
 * mm_colsum_multi_ws_len(segs, nseg) floats.  mm_wsum_multi: nseg <= 16 sums
 * out [n] = sum over s < S of x[s n + e] in mm_gemm_wgrad's reduction order. */
typedef struct {
    const float* x;
    long R;
    int N;
    float* out;
} mm_colsum_seg_t;
typedef struct {
    const float* x;
    long n;
    int S;
    float* out;
} mm_wsum_seg_t;
long mm_colsum_multi_ws_len(const mm_colsum_seg_t* segs, int nseg);
int mm_colsum_multi(const mm_colsum_seg_t* segs, int nseg, float* ws, void* stream);
int mm_wsum_multi(const mm_wsum_seg_t* segs, int nseg, void* stream);
int mm_mse_loss_partials(int M);
int mm_mse_loss(const float* v, const float* rtg, int M, float* dv, float* partial, void* stream);
int mm_losses_final(const float* ppo_partial, int n_ppo, const float* mse_partial, int n_mse, int M, float* out,
                    void* stream);

/* clip_grad_norm_(params, max_norm) followed by Adam.step() (PPO.py:74-85),
 * for up to 4 networks ("segments") at once, each over flat f32 buffers of n
 * elements: param, grad, exp_avg, exp_avg_sq.  Per segment the gradient is
 * first scaled, g0 = grad_scale * grad (1 / world after a data-parallel
 * all-reduce of sums; 1.0 otherwise), the L2 norm of g0 (fp64 partial sums,
 * fixed order) gives coef = min(1, max_norm / (norm + 1e-6)) (max_norm <= 0:
 * no clipping), then torch.optim.Adam's rule on g = coef * g0: exp_avg += (1 - beta1) (g - exp_avg); exp_avg_sq = exp_avg_sq
 * beta2 + (1 - beta2) g g; param += -step_size exp_avg / (sqrt(exp_avg_sq) /
 * bc2_sqrt + eps), with step_size = lr / (1 - beta1^t) and bc2_sqrt =
 * sqrt(1 - beta2^t) formed by the caller for step t.  grad is not modified.
 * norms [nseg] (may be NULL) receives each segment's norm before clipping
 * (clip_grad_norm_'s return value).  ws: mm_clip_adam_ws_len(nseg) floats,
 * 8-byte aligned. */
typedef struct {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    long n;
    float max_norm;
    float step_size;
    float bc2_sqrt;
    float grad_scale;
} mm_adam_seg_t;
long mm_clip_adam_ws_len(int nseg);
int mm_clip_adam(const mm_adam_seg_t* segs, int nseg, float beta1, float beta2, float eps, float* ws, float* norms,
                 void* stream);

/* The actor's two heads fused with mm_sample: logits =
 * h W^T + b for the concatenated heads W = [move_head.weight; mark_head.weight]
 * [6, K] and b [6] (networks.py:38-41), then the draw of mm_sample with the
 * same Philox counters (seed, offset, row).  h [M, ldh] f32 is the last hidden
 * layer (K % 4 == 0, K <= 1024, 16-byte aligned rows).  logits [M, 6] may be
 * NULL (it receives the 5 move logits and the mark logit when given). */
int mm_head_sample(const float* h, int ldh, int K, const float* w, const float* b, const uint8_t* masks, int M,
                   uint64_t seed, uint64_t offset, int8_t* actions, float* logp, float* joint_logp, float* logits,
                   void* stream);
/* mm_head_sample whose Philox counter offset is offset + *offset_dev (offset_dev a
 * device uint64, may be NULL): a captured HIP graph of the rollout bakes the
 * host argument in, so each replay reads its base offset from the device and
 * advances it there -- the same draws as the uncaptured rollout. */
int mm_head_sample_ex(const float* h, int ldh, int K, const float* w, const float* b, const uint8_t* masks, int M,
                      uint64_t seed, uint64_t offset, const uint64_t* offset_dev, int8_t* actions, float* logp,
                      float* joint_logp, float* logits, void* stream);

/* The heads alone (the update's forward; networks.py:38-41): logits [M, 6] =
 * h W^T + b with mm_head_sample's arithmetic per row, so the logits equal the
 * ones mm_head_sample computes for the same rows.  Same operand rules (K % 4 ==
 * 0, K <= 1024, 16-byte aligned rows); M * ldh * 4 < 2^31. */
int mm_heads_fwd(const float* h, int ldh, int K, const float* w, const float* b, int M, float* logits, void* stream);

/* The critic's value in one launch (networks.py:87-102, inference: PPO.get_batch's per-step
 * self.critic(obs), PPO.py:111): v [M] = w2 . ReLU(w1 ReLU(w0 x + b0) + b1) + b2 for x [M, K0] (row
 * stride ldx), w0 [H0, K0], w1 [H1, H0], w2 [1, H1] (nn.Linear layouts), on the fp32 MFMA (exact fmaf
 * chains, fp32 accumulation).  K0 <= 132, H0 = H1 = 64 (PPO's Critic); other shapes return MM_E_ARG. */
int mm_critic_value(const float* x, int ldx, int K0, int M, int H0, int H1, const float* w0, const float* b0,
                    const float* w1, const float* b1, const float* w2, const float* b2, float* v, void* stream);

/* Actor front-end, fused (networks.py:31-34,51-82): the 23 feature embeddings
 * (Projection; parity != 0 keeps quirk Q1, every embedding reads x[:, 0:d_i]),
 * Q/K/V, softmax(QK^T/sqrt(10))V and the residual.
 *
 * mm_actor_front_prep: builds the workspace ws [mm_actor_front_ws_len()] from
 * the parameters -- wproj/bproj: HOST arrays of the 23 device pointers of
 * projection.layers[i].weight [20, d_i] / .bias [20]; wq/wk [10,20], wv
 * [20,20] (nn.Linear layout).  Call again whenever the parameters change.
 * mm_actor_front_fwd: h [B, 460] f32 for B rows of x [B, ldx] (ldx >= 65). */
int mm_actor_front_ws_len(void);
int mm_actor_front_prep(const float* const* wproj, const float* const* bproj, const float* wq, const float* wk,
                        const float* wv, float* ws, void* stream);
int mm_actor_front_fwd(const float* ws, const float* x, int ldx, int B, int parity, float* h, void* stream);

/* mm_actor_front_fwd with the kernel chosen by `algo`:
 * MM_FRONT_FWD_ROW1 (mm_actor_front_fwd's): one query row per lane;
 * MM_FRONT_FWD_ROW2: two query rows per lane, each k_j / v_j LDS read feeding
 * both (half the K/V LDS reads per sample; bit-identical to ROW1);
 * MM_FRONT_FWD_MFMA: the two attention products on the fp32 MFMA (fp32 fmaf
 * chains in another summation order: within fp32 rounding of ROW1, not
 * bit-identical to it). */
#define MM_FRONT_FWD_ROW1 0
#define MM_FRONT_FWD_ROW2 1
#define MM_FRONT_FWD_MFMA 2
int mm_actor_front_fwd_ex(const float* ws, const float* x, int ldx, int B, int parity, float* h, int algo,
                          void* stream);

/* Backward of mm_actor_front_fwd for the upstream gradient dh [B, 460]: a
 * persistent grid of `grid` workgroups (2 per CU is the design point), each
 * writing one row of partial [grid, mm_actor_front_partial_len()]; the rows
 * are then summed in fp64 into red (8-byte aligned, room for
 * 2 x mm_actor_front_partial_len() floats = that many doubles) and turned into
 * grad [mm_actor_front_grad_len()] = [dwq 10x20 | dwk 10x20 | dwv 20x20 |
 * dwp 23x20x4 (embedding i's weight gradient zero-padded to 4 inputs) |
 * dbp 23x20].  Every sum has a fixed order (deterministic). */
int mm_actor_front_grad_len(void);
int mm_actor_front_partial_len(void);
int mm_actor_front_bwd(const float* ws, const float* x, int ldx, int B, int parity, const float* dh, float* partial,
                       int grid, float* red, float* grad, void* stream);
/* mm_actor_front_bwd with the attention backward's algorithm chosen:
 * MM_FRONT_BWD_VALU (mm_actor_front_bwd's): fp32 FMA, one lane per token;
 * MM_FRONT_BWD_MFMA: the per-sample products S = QK^T, dP = dctx V^T, dV, dK,
 * dQ on the fp32 MFMA (v_mfma_f32_16x16x4_f32, exact fmaf chains; the faster:
 * 1.22 vs 1.59 ms at 419,430 rows; `grid` from mm_actor_front_bwd_grid).  Same outputs and
 * partial layout; sums in a fixed order either way. */
#define MM_FRONT_BWD_MFMA 0
#define MM_FRONT_BWD_VALU 1
int mm_actor_front_bwd_ex(const float* ws, const float* x, int ldx, int B, int parity, const float* dh,
                          float* partial, int grid, float* red, float* grad, int algo, void* stream);
/* The persistent grid to pass as `grid` for B samples and `algo` (this build's
 * workgroup shape and workgroups per CU of the current device), or MM_E_ARG. */
int mm_actor_front_bwd_grid(int B, int algo);
/* mm_actor_front_bwd_ex writing each parameter gradient straight into its
 * own buffer in the module's layout (the update's .grad storage): wproj_grad /
 * bproj_grad are HOST arrays of the 23 device pointers of the gradients of
 * projection.layers[i].weight [20, d_i] / .bias [20]; wq_grad, wk_grad [10, 20],
 * wv_grad [20, 20]. */
int mm_actor_front_bwd_to(const float* ws, const float* x, int ldx, int B, int parity, const float* dh,
                          float* partial, int grid, float* red, float* const* wproj_grad, float* const* bproj_grad,
                          float* wq_grad, float* wk_grad, float* wv_grad, int algo, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MARLMAZE_H */
