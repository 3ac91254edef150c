// stencilx.h -- the rotating-ring sweep with shared block starts.
//
// Same cell arithmetic and register pipeline as stencild.h (a wave = a
// 256-column window walking a row block, float4 per lane, W/E by DPP, the
// rotating two-row ring of 2K + D + 1 float4, scaled levels under an
// exactness guard); what changes is how row blocks begin.
//
// In stencild.h every block walks the light cone of its first output row
// before it: K input rows of its upper neighbour and K (K - 1) / 2 row-levels
// that the neighbour evaluates too (at 8192^2, K = 20: ~155-row blocks read
// 1.26x their rows and evaluate 1.13x their row-levels, half of it at each
// end).  Here the blocks of a strip come in PAIRS that start at a shared
// boundary and walk away from it -- the upper one up, the lower one down --
// in two waves of one workgroup.  Level l of either first row needs level
// l - 1 of the other's first row, which the other has just formed: at step
// l + 1 each wave takes that row from its partner through LDS (into the
// A_{l-1} register of the ring) and publishes its own level l.  The
// prologue is K + 2 steps instead of 2K + 1, loads one row of the partner
// instead of K, and evaluates no row-level twice.  The walk's other end
// keeps stencild.h's run-on past the block (a boundary where two walks end
// would need the ring live out of the unrolled loop at every exit: the
// register allocator spills the ring).  A strip is two cone-start blocks
// (the top one walks down, the bottom one up: their global edge row is then
// their first output row, copied in the prologue as in stencild.h) and
// pairs between them; a pair's rows are the two waves of one workgroup.
//
// The exchange is wave to wave through LDS, a flag per direction and two
// slots (no barrier); a round is consumed one level step after it is
// published, so the partner's write is normally long done.
//
// Walking up costs the same as walking down here: the upward step forms
// ((S + W) + E) in temporaries with the DPP moves fused into the adds, as the
// downward one does, and only the final packed + N lands in place in S.
//
// Exactness guard: a paired wave's results depend on its partner's inputs,
// so the scaled walk stands only if no wave of the workgroup saw an input
// outside the range; otherwise all of them walk again with the exact
// arithmetic (one barrier at the end of the scaled walk).
#pragma once

#include "stencild.h"  // smi_amd/csrc (the harness builds with -I smi_amd/csrc)

namespace smi {

// Launch geometry: strips as SweepDGeom; every strip cut into an even
// number of blocks (nb interior strips, nb_ce edge-column strips): the top
// and bottom blocks walk a cone at their start, the others in start-sharing
// pairs.  A block's rows are in proportion to its weight in 16ths (16 for a
// paired block, wcone for the two cone-start blocks: their cone's extra rows
// and levels make them shorter).
struct SweepXGeom {
    int nstrips, n_int, int0;
    int ce[4];
    int nb, nb_ce;  // blocks per interior / edge-column strip (even, >= 2)
    int wcone;      // weight of a cone-start block (16ths)
    int tasks;      // waves = n_int * nb + (edge-column strips) * nb_ce
};

// LDS of one workgroup: per wave its outbox towards the partner (two slots
// of one float4 per lane) and the round flag; the workgroup's guard verdicts.
struct SweepXShared {
    float4 box[4][2][64];  // [wave][slot][lane]
    int flag[4];           // rounds published by the wave
    int bad[4];
};

// The waves of a strip (offset k of nbs) and its blocks: k < nbs - 2 are the
// pairs (k even: block k + 1, walking up; k odd: block k + 1, walking down;
// the pair starts at the boundary between them), k = nbs - 2 the top block
// (down), k = nbs - 1 the bottom block (up).
__host__ __device__ inline int sweepx_block_of(int k, int nbs) {
    return k < nbs - 2 ? k + 1 : (k == nbs - 2 ? 0 : nbs - 1);
}

// Rows [o0, o1) of block b: out_rows split in proportion to the weights
// (blocks 0 and nbs - 1: wcone, the others 16); integer arithmetic, so both
// neighbours of a boundary compute it alike.
__host__ __device__ inline void sweepx_block_rows(int row_lo, int row_hi, int b, int nbs, int wcone, int *o0,
                                                  int *o1) {
    const long tot = (long)(nbs - 2) * 16 + 2L * wcone;
    const long pre = b == 0 ? 0 : wcone + (long)(b - 1) * 16;
    const long wb = (b == 0 || b == nbs - 1) ? wcone : 16;
    const long out_rows = row_hi - row_lo;
    *o0 = row_lo + (int)(out_rows * pre / tot);
    *o1 = b == nbs - 1 ? row_hi : row_lo + (int)(out_rows * (pre + wb) / tot);
}

template <int K>
struct SweepX {
    static_assert(K >= 3 && K <= 24, "3 <= K <= 24");
    using Geom = DeepGeom<K>;
    static constexpr int LL = Geom::LL;
    static constexpr int KC = 4 * LL;
    static constexpr int D = Geom::D;
    static constexpr int N = 2 * K + D + 1;  // ring positions = rows per loop body
    static constexpr int PRO = 2 * K + 1;    // cone prologue rows
    static constexpr int PROX = K + 2;       // paired prologue rows
    static constexpr int J0 = PRO % N;       // ring rotation at the steady loop's start
    static constexpr int G = 2;              // rows per end-of-walk check (stencild.h)
    static_assert(N % G == 0, "the loop body must hold whole groups");
    static_assert(KC >= K, "apron narrower than the cone");
    static constexpr int kExpLo = 2 * K - 124, kExpHi = 126 - 2 * K;
    static constexpr float kUnscale = 1.0f / (float)(1ull << (2 * K));

    const float *__restrict__ in;
    float *__restrict__ out;
    int rows, cols;
    int o0, o1;
    int r_begin;    // input row of step 0
    int n_in;       // input rows walked (steps 0 .. n_in - 1)
    int voff_ld, voff, row_bytes;
    unsigned long long maskL, maskR, maskE;
    f32x2 quarter;
    int emin, emax;
    SweepXShared *sh;
    int wv, ps;          // my wave and my partner's in the workgroup
    int r_out, r_in;     // rounds published / consumed
    int lane;
    int prio_phase;  // SMI_X_PRIO_ROWS experiment
    float4 R[N];

    static constexpr int ph(int p, int j) { return ((p - j) % N + N) % N; }

    template <bool REV>
    __device__ __forceinline__ float4 ld(int t) const {
#ifdef SMI_X_NOMEM  // experiment: levels only, no loads (timing)
        const float f = (float)(t & 7) * 0.125f + (float)voff_ld * 1e-6f;
        return make_float4(f, f + 0.25f, f + 0.5f, f + 0.75f);
#endif
#ifdef SMI_X_CACHED  // experiment: every load hits one of two cache-resident rows, no stores (VALU timing)
        const int r = __builtin_amdgcn_readfirstlane(t & 1);
#else
        const int r = __builtin_amdgcn_readfirstlane(min(max(REV ? r_begin - t : r_begin + t, 0), rows - 1));
#endif
        const char *rowp = reinterpret_cast<const char *>(in + (size_t)r * cols);
        return *reinterpret_cast<const float4 *>(rowp + (unsigned)voff_ld);
    }

    __device__ __forceinline__ void note(const float4 &x) {
        const int e0 = __builtin_amdgcn_frexp_expf(x.x), e1 = __builtin_amdgcn_frexp_expf(x.y);
        const int e2 = __builtin_amdgcn_frexp_expf(x.z), e3 = __builtin_amdgcn_frexp_expf(x.w);
        emin = min(emin, min(e0, e1));
        emax = max(emax, max(e0, e1));
        emin = min(emin, min(e2, e3));
        emax = max(emax, max(e2, e3));
        asm("" : "+v"(emin), "+v"(emax));  // folded row by row (see stencild.h)
    }

    // One level step of 4 cells per lane, ((S + W) + E) + N, the result in
    // the registers of the older operand row (tied asm operands).  Walking
    // down the older row is N: (S + W) + E in temporaries, the packed + N in
    // place.  Walking up the older row is S: (S + W) + E again in
    // temporaries (the DPP moves fused into the adds by the compiler), and
    // the packed + N writes S's registers.
    template <bool REV, int CE, bool SC>
    __device__ __forceinline__ float4 step(const float4 &older, const float4 &c, const float4 &nw) const {
        const float4 &s = REV ? older : nw;
        const float w = shr1_any(c.w);
        const float e = shl1_any(c.x);
        float b0 = __fadd_rn(__fadd_rn(s.x, w), c.y);
        float b1 = __fadd_rn(__fadd_rn(s.y, c.x), c.z);
        float b2 = __fadd_rn(__fadd_rn(s.z, c.y), c.w);
        float b3 = __fadd_rn(__fadd_rn(s.w, c.z), e);
        asm("" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));  // no re-pairing into packed adds with moves
        f32x2 o01 = f32x2{older.x, older.y};
        f32x2 o23 = f32x2{older.z, older.w};
        if constexpr (!REV) {
            asm("v_pk_add_f32 %0, %1, %0" : "+v"(o01) : "v"(f32x2{b0, b1}));
            asm("v_pk_add_f32 %0, %1, %0" : "+v"(o23) : "v"(f32x2{b2, b3}));
        } else {
            asm("v_pk_add_f32 %0, %1, %2" : "+v"(o01) : "v"(f32x2{b0, b1}), "v"(f32x2{nw.x, nw.y}));
            asm("v_pk_add_f32 %0, %1, %2" : "+v"(o23) : "v"(f32x2{b2, b3}), "v"(f32x2{nw.z, nw.w}));
        }
        if constexpr (!SC) {
            asm("v_pk_mul_f32 %0, %0, %1" : "+v"(o01) : "v"(quarter));
            asm("v_pk_mul_f32 %0, %0, %1" : "+v"(o23) : "v"(quarter));
        }
        float4 o = make_float4(o01.x, o01.y, o23.x, o23.y);
        if constexpr (CE & 1) {
            const float cx = SC ? c.x * 4.0f : c.x;
            asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(o.x) : "v"(cx), "s"(maskL));
        }
        if constexpr (CE & 2) {
            const float cw = SC ? c.w * 4.0f : c.w;
            asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(o.w) : "v"(cw), "s"(maskR));
        }
        return o;
    }

    // level K of step t lands on row r_begin -+ (t - K)
    template <bool REV, bool SC>
    __device__ __forceinline__ void store_row(int t, const float4 &vs) const {
        float4 v = vs;
        if constexpr (SC) {
            const f32x2 q = {kUnscale, kUnscale};
            const f32x2 a = f32x2{vs.x, vs.y} * q, b = f32x2{vs.z, vs.w} * q;
            v = make_float4(a.x, a.y, b.x, b.y);
        }
        const int j = REV ? r_begin - (t - K) : r_begin + (t - K);
#ifdef SMI_X_NOMEM  // experiment: no stores either (one lane's sum keeps the levels live)
        if (j == -12345) out[lane] = v.x + v.y + v.z + v.w;
        return;
#endif
#ifdef SMI_X_CACHED
        const bool in_block = false;
#else
        const bool in_block = j >= o0 && j < o1;
#endif
        const int jj = __builtin_amdgcn_readfirstlane(min(max(j, 0), rows - 1));
        const int nrec = __builtin_amdgcn_readfirstlane(in_block ? row_bytes : 0);
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + (size_t)jj * cols, (short)0, nrec, 0x00020000);
        const u32x4 d = {__builtin_bit_cast(unsigned int, v.x), __builtin_bit_cast(unsigned int, v.y),
                         __builtin_bit_cast(unsigned int, v.z), __builtin_bit_cast(unsigned int, v.w)};
#ifdef SMI_X_STORE_AUX
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff, 0, SMI_X_STORE_AUX);
#else
        __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff, 0, 2 /* nt */);
#endif
    }

    // publish: my row into slot (round - 1) & 1 of my outbox, then (after
    // the row's write has completed) the round number
    __device__ __forceinline__ void publish(const float4 &v) {
        ++r_out;
        sh->box[wv][(r_out - 1) & 1][lane] = v;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        *reinterpret_cast<volatile int *>(&sh->flag[wv]) = r_out;
    }
    // take: wait until the partner has published this round, read its row.
    // Double buffering is safe: the partner publishes round r + 2 only after
    // taking my round r + 1, which I publish after reading its round r.
    __device__ __forceinline__ float4 take() {
        ++r_in;
        while (__builtin_amdgcn_readfirstlane(*reinterpret_cast<volatile int *>(&sh->flag[ps])) < r_in)
            __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        return sh->box[ps][(r_in - 1) & 1][lane];
    }

    // A steady-state / cone-prologue step: as SweepD::row (TC >= 0: the cone
    // prologue's compile-time t, level l from t >= 2l, the global edge row
    // copied where t - l == K).
    template <bool REV, int CE, bool SC, int J, int TC>
    __device__ __forceinline__ void row(int t) {
        R[ph(0, J)] = ld<REV>(min(t + D, n_in - 1));
        const float4 x = R[ph(D, J)];
        if constexpr (SC) note(x);
        float4 v = x;
#ifdef SMI_X_NOLEVELS  // experiment: loads and stores only (timing)
        if constexpr (TC < 0 || TC == 2 * K) store_row<REV, SC>(t, v);
        return;
#endif
#ifdef SMI_X_LANEMASK
        // experiment: level l needs lanes [m, 64 - m), m = (l - 1) / 4 (the
        // cone's valid columns plus the lanes their DPP reads come from);
        // the rest run with EXEC off (a lane-op and its register reads saved)
        if constexpr (TC < 0) {
            static_assert(K % 4 == 0, "lane-mask groups of 4 levels");
            static_for<K / 4>([&](auto M) {
                constexpr int m = M;
                if (m == 0 || (lane >= m && lane < 64 - m)) {
                    static_for<4>([&](auto L4) {
                        constexpr int l = 4 * m + L4 + 1;
                        constexpr int ia = ph(D + 2 * l, J), ib = ph(D + 2 * l - 1, J);
                        float4 nv = step<REV, CE, SC>(R[ia], R[ib], v);
                        if constexpr (l < K) R[ia] = nv;
                        v = nv;
                    });
                }
            });
            store_row<REV, SC>(t, v);
            return;
        }
#endif
        static_for<K>([&](auto L) {
            constexpr int l = L + 1;
            if constexpr (TC < 0 || TC >= 2 * l) {
                constexpr int ia = ph(D + 2 * l, J), ib = ph(D + 2 * l - 1, J);
                const float4 older = R[ia], mid = R[ib];
                float4 nv = step<REV, CE, SC>(older, mid, v);
                if constexpr (TC >= 0 && TC - l == K) {
                    const float4 m = SC ? make_float4(mid.x * 4.0f, mid.y * 4.0f, mid.z * 4.0f, mid.w * 4.0f) : mid;
                    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.x) : "v"(m.x), "s"(maskE));
                    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.y) : "v"(m.y), "s"(maskE));
                    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.z) : "v"(m.z), "s"(maskE));
                    asm("v_cndmask_b32 %0, %0, %1, %2" : "+v"(nv.w) : "v"(m.w), "s"(maskE));
                }
                if constexpr (l < K) R[ia] = nv;
                v = nv;
            }
        });
        if constexpr (TC < 0 || TC == 2 * K) store_row<REV, SC>(t, v);
    }

    // Paired prologue step TC (compile-time, TC = t): input row 0 is the
    // partner's first row.  Level l is formed from step l + 1 on (my rows
    // only); at step l + 1 its older operand A_{l-1} -- level l - 1 of the
    // partner's first row -- comes from the partner (l >= 2; for l = 1 it is
    // the loaded row 0), and the level-l row just formed (my first row) is
    // published for the partner's step l + 2.
    template <bool REV, int CE, bool SC, int J, int TC>
    __device__ __forceinline__ void rowx(int t) {
        R[ph(0, J)] = ld<REV>(min(t + D, n_in - 1));
        const float4 x = R[ph(D, J)];
        if constexpr (SC) note(x);
        float4 v = x;
        static_for<K>([&](auto L) {
            constexpr int l = L + 1;
            if constexpr (TC >= l + 1) {
                constexpr int ia = ph(D + 2 * l, J), ib = ph(D + 2 * l - 1, J);
                if constexpr (TC == l + 1 && l >= 2) R[ia] = take();
                float4 nv = step<REV, CE, SC>(R[ia], R[ib], v);
                if constexpr (l < K) R[ia] = nv;
                v = nv;
                if constexpr (TC == l + 1 && l < K) publish(nv);
            }
        });
        if constexpr (TC == K + 1) store_row<REV, SC>(t, v);
    }

    // Level l of the row at rotation J (steady state): v = new_{l-1} in, new_l out.
    template <bool REV, int CE, bool SC, int J, int l>
    __device__ __forceinline__ void level(float4 &v) {
        constexpr int ia = ph(D + 2 * l, J), ib = ph(D + 2 * l - 1, J);
        float4 nv = step<REV, CE, SC>(R[ia], R[ib], v);
        if constexpr (l < K) R[ia] = nv;
        v = nv;
    }

    // Steady-state rows t and t + 1 (rotations J, J + 1), their level chains
    // interleaved one level apart (stencild.h SweepD::pair): row t + 1's
    // level l - 1 needs row t's level l - 2 only, so each pair of level
    // steps is independent -- twice the independent work per wave.
    template <bool REV, int CE, bool SC, int J>
    __device__ __forceinline__ void pairrows(int t) {
        R[ph(0, J)] = ld<REV>(min(t + D, n_in - 1));
        float4 va = R[ph(D, J)];
        float4 vb = R[ph(D, J + 1)];
        if constexpr (SC) {
            note(va);
            note(vb);
        }
        level<REV, CE, SC, J, 1>(va);
        static_for<K - 1>([&](auto L) {
            constexpr int l = L + 2;
            level<REV, CE, SC, J, l>(va);
            level<REV, CE, SC, (J + 1) % N, l - 1>(vb);
        });
        store_row<REV, SC>(t, va);
        R[ph(0, J + 1)] = ld<REV>(min(t + 1 + D, n_in - 1));
        level<REV, CE, SC, (J + 1) % N, K>(vb);
        store_row<REV, SC>(t + 1, vb);
    }

    // rows t + r .. t + N - 1 of one loop body (stencild.h SweepD::body)
    template <bool REV, int CE, bool SC, int r>
    __device__ __forceinline__ bool body(int t) {
        if constexpr (r == N) {
            return true;
        } else {
#ifdef SMI_X_PAIRROWS
            static_assert(N % 2 == 0 && G == 2, "pairs of rows need an even cycle");
            if (t + r >= n_in) return false;
            pairrows<REV, CE, SC, (J0 + r) % N>(t + r);
            return body<REV, CE, SC, r + 2>(t);
#else
            if constexpr (r % G == 0) {
                if (t + r >= n_in) return false;
#ifdef SMI_X_PRIO_ROWS
                // experiment: the two waves of a SIMD trade the VALU issue
                // priority every SMI_X_PRIO_ROWS rows, in opposite phase
                // (otherwise the older wave wins every arbitration and the
                // younger one finishes alone, at the one-wave issue rate)
                if ((((t + r) / SMI_X_PRIO_ROWS) + prio_phase) & 1)
                    __builtin_amdgcn_s_setprio(1);
                else
                    __builtin_amdgcn_s_setprio(0);
#endif
            }
            row<REV, CE, SC, (J0 + r) % N, -1>(t + r);
            return body<REV, CE, SC, r + 1>(t);
#endif
        }
    }

    template <bool REV, int CE, bool SC>
    __device__ __forceinline__ bool run(bool paired) {
        emin = 0;
        emax = 0;
        int t;
        if (paired) {
            // rows 0 .. D-1 into position 0 of rotations K - 1 - D + d; the
            // K + 2 prologue steps run at rotations K - 1 .. 2K, so the loop
            // starts at rotation 2K + 1 = PRO (mod N) as after a cone prologue
            static_for<D>([&](auto Dd) {
                constexpr int d = Dd;
                R[ph(0, d - D + K - 1)] = ld<REV>(d);
            });
            static_for<PROX>([&](auto T) {
                constexpr int tc = T;
                if constexpr (tc % G == 0 && tc > 0) __builtin_amdgcn_sched_barrier(0);
                rowx<REV, CE, SC, (tc + K - 1) % N, tc>(tc);
            });
            t = PROX;
        } else {
            static_for<D>([&](auto Dd) {
                constexpr int d = Dd;
                R[ph(0, d - D)] = ld<REV>(d);
            });
            static_for<PRO>([&](auto T) {
                constexpr int tc = T;
                if constexpr (tc % G == 0 && tc > 0) __builtin_amdgcn_sched_barrier(0);
                row<REV, CE, SC, tc % N, tc>(tc);
            });
            t = PRO;
        }
        for (;; t += N)
            if (!body<REV, CE, SC, 0>(t)) break;
        if constexpr (SC) return emin < kExpLo || emax > kExpHi;
        return false;
    }

    template <bool REV, int CE>
    __device__ __forceinline__ void go(bool paired) {
        const bool bad = __builtin_amdgcn_ballot_w64(run<REV, CE, true>(paired)) != 0;
#ifdef SMI_X_NOBARRIER
        if (!bad) return;
        __builtin_amdgcn_s_waitcnt(0x0F70);
        run<REV, CE, false>(paired);
        return;
#endif
        // the scaled walk stands only if no wave of the workgroup saw an
        // input outside the guard's range (paired waves' results depend on
        // each other's inputs)
        if (lane == 0) sh->bad[wv] = bad;
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(sh->bad[0] | sh->bad[1] | sh->bad[2] | sh->bad[3])) return;
        __builtin_amdgcn_s_waitcnt(0x0F70);  // the exact walk's stores land after these
        run<REV, CE, false>(paired);
    }
};

// Wave order: pair-band major, like stencild.h's row-band order -- waves
// 2i, 2i + 1 are one pair (or the top and bottom blocks: "pair" nbs/2 - 1)
// of one strip; consecutive pairs are the same band of neighbouring strips
// (interior strips, then the edge-column strips with their own bands), so a
// workgroup holds one band of two neighbouring strips and an XCD's
// contiguous workgroups hold whole row bands: the strips' overlapping
// window columns meet in its L2.
#ifdef SMI_X_WAVETIMES
// experiment: per wave, its hardware place and its start / end shader clock
__device__ unsigned long long *g_wavetimes;
#endif

template <int K>
__device__ __forceinline__ void sweepx_wave(const SweepKArgs &a, const SweepXGeom &g, SweepXShared *sh, int gb,
                                            int wv, int lane) {
    using S = SweepX<K>;
    constexpr int SW = 256 - 2 * S::KC;
    const int ti = g.n_int * g.nb;
    int strip, k, nbs;
    if (gb < ti) {
        const int pr = gb >> 1, band = pr / g.n_int;
        strip = g.int0 + (pr - band * g.n_int);
        k = 2 * band + (gb & 1);
        nbs = g.nb;
    } else {
        int nce = 0;
        while (nce < 4 && g.ce[nce] >= 0) ++nce;
        const int pr = (gb - ti) >> 1, band = pr / nce;
        strip = g.ce[pr - band * nce];
        k = 2 * band + (gb & 1);
        nbs = g.nb_ce;
    }
    const int b = sweepx_block_of(k, nbs);
    S w;
    w.in = a.in;
    w.out = a.out;
    w.rows = a.rows;
    w.cols = a.cols;
    w.sh = sh;
    w.wv = wv;
    w.ps = wv ^ 1;
    w.r_out = w.r_in = 0;
    w.lane = lane;
#if defined(SMI_X_PRIO_BLOCK)
    w.prio_phase = __builtin_amdgcn_readfirstlane((int)(blockIdx.x >> 8) & 1);
#else
    // HW_ID bits [3:0]: this wave's slot on its SIMD (s_getreg hwreg(HW_REG_HW_ID, 0, 4))
    w.prio_phase = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 4) & 1);
#endif
    sweepx_block_rows(a.row_lo, a.row_hi, b, nbs, g.wcone, &w.o0, &w.o1);
#ifdef SMI_X_NOPAIR
    const bool paired = false;
#else
    const bool paired = k < nbs - 2;
#endif
    const bool rev = b & 1;  // odd blocks (the upper block of a pair, the bottom block) walk up
    const int cs = (a.col_lo & ~31) + strip * SW;
    const int cb = cs - S::KC + 4 * lane;
    w.voff_ld = min(max(cb, 0), a.cols - 4) * 4;
    const bool st = lane >= S::LL && lane < 64 - S::LL && cb >= a.col_lo && cb < a.col_hi;
    w.row_bytes = a.cols * 4;
    w.voff = st ? cb * 4 : 0x7ffffff0;
    w.maskL = __builtin_amdgcn_ballot_w64(a.gL && cb == 0);
    w.maskR = __builtin_amdgcn_ballot_w64(a.gR && cb + 4 == a.cols);
    w.quarter = f32x2{0.25f, 0.25f};
    const int ce = ((a.gL && cs - S::KC <= 0) ? 1 : 0) | ((a.gR && cs - S::KC + 256 >= a.cols) ? 2 : 0);
    // a global edge row is the first output row of a cone-start walk (the
    // top block walks down from row 0, the bottom block up from row X-1)
    const bool top = a.gT && b == 0;
    const bool bot = a.gB && b == nbs - 1;
    w.maskE = __builtin_amdgcn_ballot_w64(top || bot);
    const int s0 = paired ? 1 : K;
    w.r_begin = rev ? w.o1 - 1 + s0 : w.o0 - s0;
    w.n_in = s0 + (w.o1 - w.o0) + K;
    switch ((rev ? 2 : 0) + (ce ? 1 : 0)) {
    case 0: w.template go<false, 0>(paired); break;
    case 1: w.template go<false, 3>(paired); break;
    case 2: w.template go<true, 0>(paired); break;
    default: w.template go<true, 3>(paired); break;
    }
}

#ifndef SMI_X_WPE
#define SMI_X_WPE 1
#endif
template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SMI_X_WPE, 8))) void sweepx_kernel(SweepKArgs a,
                                                                                               SweepXGeom g) {
    __shared__ SweepXShared sh;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int gb = lb * 4 + wv;
    if (threadIdx.x < 4) {
        sh.flag[threadIdx.x] = 0;
        sh.bad[threadIdx.x] = 0;
    }
    __syncthreads();
    if (gb < g.tasks) {
#ifdef SMI_X_WAVETIMES
        const unsigned long long t0 = __builtin_readcyclecounter();
#endif
        sweepx_wave<K>(a, g, &sh, gb, wv, lane);
#ifdef SMI_X_WAVETIMES
        const unsigned long long t1 = __builtin_readcyclecounter();
        if (lane == 0) {
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
            g_wavetimes[3 * gb + 0] = ((unsigned long long)xcc << 32) | hw;
            g_wavetimes[3 * gb + 1] = t0;
            g_wavetimes[3 * gb + 2] = t1;
        }
#endif
    } else {
        __syncthreads();  // the guard's barrier of the workgroup's walking waves
    }
}

// ---------------------------------------------------------------------------
// Experiment (SMI_X_UNEQUAL): the library's sweepd walk with unequal halves.
// With two waves per SIMD the older one (blockIdx < P: the first workgroup on
// every CU) issues at the one-wave rate and the younger one takes what is
// left, so equal blocks leave the younger wave walking alone for the last
// third of the pass (xbench_x20t wavetimes).  Here block pairs (2j, 2j+1) of
// the library geometry are one pair task: workgroup b < P (old) walks the top
// fo/256 of the pair's output rows, workgroup b + P (young) the rest.
#ifdef SMI_X_UNEQUAL
template <int K>
__device__ __forceinline__ void sweepu_task(const SweepKArgs &a, int strip, int o0, int o1, int lane) {
    using S = SweepD<K>;
    constexpr int SW = 256 - 2 * S::KC;
    S w;
    w.in = a.in;
    w.out = a.out;
    w.rows = a.rows;
    w.cols = a.cols;
    w.o0 = o0;
    w.o1 = o1;
    w.n_in = (w.o1 - w.o0) + 2 * K;
    const int cs = (a.col_lo & ~31) + strip * SW;
    const int cb = cs - S::KC + 4 * lane;
    w.voff_ld = min(max(cb, 0), a.cols - 4) * 4;
    const bool st = lane >= S::LL && lane < 64 - S::LL && cb >= a.col_lo && cb < a.col_hi;
    w.row_bytes = a.cols * 4;
    w.voff = st ? cb * 4 : 0x7ffffff0;
    w.maskL = __builtin_amdgcn_ballot_w64(a.gL && cb == 0);
    w.maskR = __builtin_amdgcn_ballot_w64(a.gR && cb + 4 == a.cols);
    w.quarter = f32x2{0.25f, 0.25f};
    const int ce = ((a.gL && cs - S::KC <= 0) ? 1 : 0) | ((a.gR && cs - S::KC + 256 >= a.cols) ? 2 : 0);
    const bool top = a.gT && w.o0 == 0;
    const bool bot = a.gB && w.o1 == a.rows;
    const bool rev = bot && !top;
    w.maskE = __builtin_amdgcn_ballot_w64(top || bot);
    w.r_begin = rev ? w.o1 - 1 + K : w.o0 - K;
    switch ((rev ? 2 : 0) + (ce ? 1 : 0)) {
    case 0: w.template go<false, 0>(); break;
    case 1: w.template go<false, 3>(); break;
    case 2: w.template go<true, 0>(); break;
    default: w.template go<true, 3>(); break;
    }
}

template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 8))) void sweepu_kernel(SweepKArgs a,
                                                                                                 SweepDGeom g,
                                                                                                 int P, int fo) {
    const int b = blockIdx.x;
    const int gen = b >= P ? 1 : 0;
    const int lp = xcd_remap(b - gen * P, P);
    const int lane = threadIdx.x & 63;
    const int pair = __builtin_amdgcn_readfirstlane(lp * 4 + (int)(threadIdx.x >> 6));
    const int pi = g.n_int * (g.nrb >> 1);
    if (pair >= (g.tasks >> 1)) return;
    int strip, rb, nb;
    if (pair < pi) {
        const int rp = pair / g.n_int;
        strip = g.int0 + pair - rp * g.n_int;
        rb = 2 * rp;
        nb = g.nrb;
    } else {
        const int t2 = pair - pi, h = g.nrb_ce >> 1;
        const int k = t2 / h;
        strip = g.ce[k];
        rb = 2 * (t2 - k * h);
        nb = g.nrb_ce;
    }
    int o0, o1, x0, x1;
    sweepd_block_rows(a, rb, nb, g.wlast, &o0, &x0);
    sweepd_block_rows(a, rb + 1, nb, g.wlast, &x1, &o1);
    const int om = o0 + (int)((long)(o1 - o0) * fo / 256);
#ifdef SMI_X_WAVETIMES
    const unsigned long long t0 = __builtin_readcyclecounter();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#endif
    if (gen == 0) sweepu_task<K>(a, strip, o0, om, lane);
    else sweepu_task<K>(a, strip, om, o1, lane);
#ifdef SMI_X_WAVETIMES
    const unsigned long long t1 = __builtin_readcyclecounter();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        // shader clock cycles and 100 MHz real time of the walk
        const int gb = 2 * pair + gen;
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);
        g_wavetimes[5 * gb + 0] = ((unsigned long long)xcc << 32) | hw;
        g_wavetimes[5 * gb + 1] = t0;
        g_wavetimes[5 * gb + 2] = t1;
        g_wavetimes[5 * gb + 3] = r0;
        g_wavetimes[5 * gb + 4] = r1;
    }
#endif
}
#endif

}  // namespace smi
