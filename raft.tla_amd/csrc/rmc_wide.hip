// rmc_wide.hip — gfx950 kernels of the wide layout (raft_wide.h): the BFS,
// the successor listing and the random walks of models whose fields outgrow
// the packed layout (MCraft.cfg as shipped under a depth bound, Smokeraft's
// unbounded depth-100 walks).  One thread per state or behaviour; each lane
// materialises its successor (5,080 bytes, private memory), the fingerprint
// hashes the whole canonical record, and new states are inserted into the
// same kind of open-addressing HBM set as the packed kernels use.
#include <hip/hip_runtime.h>

#include "raft_wide.h"
#include "rmc_internal.h"

namespace rmc {
namespace wide {

__device__ __forceinline__ int w_insert(u64* __restrict__ table, u64 mask, const Fp& h, u32* full) {
    const TKey t = tkey(h, mask);
    const u64 key = t.v;
    u64 s = t.s0;
    for (u64 n = 0; n <= mask; ++n) {
        const u64 cur = table[s];
        if (cur == key) return 0;
        if (cur == 0) {
            const u64 prev = atomicCAS((unsigned long long*)&table[s], 0ull, (unsigned long long)key);
            if (prev == 0) return 1;
            if (prev == key) return 0;
        }
        s = (s + 1) & mask;
    }
    atomicOr(full, 1u);
    return 0;
}

__device__ __forceinline__ u64 w_wave_sum(u64 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        v += (u64)(u32)__shfl_xor((int)(u32)v, off) | ((u64)(u32)__shfl_xor((int)(u32)(v >> 32), off) << 32);
    return v;
}

// Store a new state (slot allocated by the caller) with its trace link and the
// fused invariant check.
template <class St>
__device__ __forceinline__ void w_store(const WModel& M, const WideBufs& B, u64 ni, const St& t, u64 parent,
                                        int lane) {
    wcopy_state(static_cast<St*>(B.store)[ni], t);
    B.parent[ni] = parent;
    B.act[ni] = (uint8_t)lane;
    const int v = wcheck_invariants(M, t);
    if (v) atomicMin((unsigned long long*)&B.ctr->viol, (unsigned long long)((ni << 4) | (u64)(v - 1)));
}

// Init (raft.tla:125-129) or SmokeInit's states: n staged records.
template <class St>
__global__ __launch_bounds__(256) void k_wseed(const WModel M, const WideBufs B, const St* staged, u64 n) {
    for (u64 t = (u64)blockIdx.x * 256ull + threadIdx.x; t < n; t += (u64)gridDim.x * 256ull) {
        if (!w_insert(B.table, B.tmask, wfp(staged[t], B.salt, M.S), &B.ctr->table_full)) continue;
        const u64 ni = atomicAdd((unsigned long long*)&B.ctr->count, 1ull);
        if (ni >= B.cap) {
            atomicOr(&B.ctr->overflow, 1u);
            continue;
        }
        w_store(M, B, ni, staged[t], ~0ull, 255);
    }
}

// One BFS level: every lane of every frontier state [lo, hi).  Successors
// outside the CONSTRAINT count as generated and are dropped; a successor the
// layout cannot hold in a field no CONSTRAINT bounds stops the search
// (Counters.overflow bits 8-11, the field).  Round 6: the parent's fingerprint
// once per state and each successor's from it (wfp_delta: the components the
// lane changed), the bag families walked only over the state's messages, and
// stuttering successors (the parent's fingerprint) not probed.
template <class St>
__global__ __launch_bounds__(256) void k_wexpand(const WModel M, const WideBufs B, u64 lo, u64 hi) {
    u64 gen = 0, probes = 0;
    u32 bad = 0;
    const int o7 = M.L.off[7];
    for (u64 i = lo + (u64)blockIdx.x * 256ull + threadIdx.x; i < hi; i += (u64)gridDim.x * 256ull) {
        St s, t;
        wcopy_state(s, static_cast<const St*>(B.store)[i]);
        const Fp h0 = wfp(s, B.salt, M.S);
        u32 g = 0;
        // lanes of families 0-6, then the three bag families over slots [0, nmsg)
        const int nb = s.nmsg, nl = o7 + 3 * nb;
        for (int q = 0; q < nl; ++q) {
            const int lane = q < o7 ? q : M.L.off[7 + (q - o7) / nb] + (q - o7) % nb;
            WDelta dl;
            const int r = wlane(M, s, lane, &t, false, &dl);
            if (r == W_OFF) continue;
            ++g;
            if (r != W_ON) {  // beyond the layout: an error for a field no CONSTRAINT bounds,
                bad |= (u32)(woverflow_bits(r) & M.unbounded);  // else beyond its bound (filtered)
                continue;
            }
            if (!win_model(M, t)) continue;
            const Fp h = wfp_delta(s, t, h0, dl, B.salt);
            if (h.k == h0.k && h.s == h0.s) continue;  // a stutter (or a full-fingerprint twin of the parent)
            ++probes;
            if (!w_insert(B.table, B.tmask, h, &B.ctr->table_full)) continue;
            const u64 ni = atomicAdd((unsigned long long*)&B.ctr->count, 1ull);
            if (ni >= B.cap) {
                atomicOr(&B.ctr->overflow, 1u);
                continue;
            }
            w_store(M, B, ni, t, i, lane);
        }
        if (g == 0) atomicMin((unsigned long long*)&B.ctr->deadlock, (unsigned long long)i);
        gen += g;
    }
    gen = w_wave_sum(gen);
    probes = w_wave_sum(probes);
    if (__lane_id() == 0 && gen) atomicAdd((unsigned long long*)&B.ctr->generated, (unsigned long long)gen);
    if (__lane_id() == 0 && probes) atomicAdd((unsigned long long*)&B.ctr->probes, (unsigned long long)probes);
    if (bad) atomicOr(&B.ctr->overflow, bad << 8);
}

// Every enabled lane of n given states, without dedup (rmc_expand).
__global__ __launch_bounds__(64) void k_wlist(const WModel M, const WState* in, u64 n, WSucc* out, u64 cap,
                                             unsigned long long* count, u64 salt) {
    const u64 p = (u64)blockIdx.x * 64ull + threadIdx.x;
    if (p >= n) return;
    WState t;
    for (int lane = 0; lane < M.L.off[10]; ++lane) {
        const int r = wlane(M, in[p], lane, &t);
        if (r == W_OFF) continue;
        const u64 o = atomicAdd(count, 1ull);
        if (o >= cap) continue;
        WSucc& w = out[o];
        w.parent = p;
        w.lane = lane;
        w.code = r;
        const int inm = r == W_ON && win_model(M, t);
        w.in_model = inm;
        w.fp = inm ? wfp(t, salt, M.S).k : 0ull;
        if (inm) wcopy_state(w.state, t);
        else wzero(&w.state, (int)sizeof(WState));
    }
}


// ---- one wave on one record in LDS (k_wsimulate_w) ----------------------------------
// Every lane of the wave calls these with the same arguments; lane q handles
// message q (KW = 64 = the wave), so a bag search is one compare per lane and a
// ballot, and an insert / removal moves every later message at once.
__device__ __forceinline__ void w_wsync() {  // the wave's LDS writes seen by the whole wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
static_assert(KW <= 64, "WaveBag: one message per lane of the wave");
struct WaveBag {
    // slot of m in the sorted bag (-1: absent); *pos = the messages below m
    static __device__ int find(const WState& s, const WMsg& m, int* pos) {
        const int ln = (int)__lane_id();
        const int n = s.nmsg;
        const int c = ln < n ? wmsg_cmp(s.msg[ln], m) : 1;
        const u64 eq = __ballot(c == 0), lt = __ballot(c < 0);
        *pos = (int)__popcll(lt);
        return eq ? (int)__builtin_ctzll(eq) : -1;
    }
    static __device__ int fits(const WState& s, const WMsg& m) {
        int pos;
        const int k = find(s, m, &pos);
        if (k >= 0) return s.cnt[k] >= CMAX ? W_DUP : W_ON;
        return s.nmsg >= KW ? W_MSGS : W_ON;
    }
    static __device__ int reply_fits(const WState& s, const WMsg& r, int x) {
        int pos;
        const int k = find(s, r, &pos);
        if (k >= 0) return s.cnt[k] >= CMAX ? W_DUP : W_ON;
        return (s.nmsg >= KW && s.cnt[x] > 1) ? W_MSGS : W_ON;
    }
    static __device__ int add(WState& s, const WMsg& m) {  // wbag_add
        const int ln = (int)__lane_id();
        w_wsync();
        int k;
        const int e = find(s, m, &k);
        const int n = s.nmsg;
        if (e >= 0) {
            const int c = s.cnt[e];
            if (c >= CMAX) return W_DUP;
            w_wsync();
            if (ln == 0) s.cnt[e] = (uint8_t)(c + 1);
            w_wsync();
            return W_ON;
        }
        if (n >= KW) return W_MSGS;
        const bool mv = ln >= k && ln < n;  // messages k .. n-1 move up one slot
        WMsg mine;
        uint8_t c = 0;
        if (mv) {
            mine = s.msg[ln];
            c = s.cnt[ln];
        }
        w_wsync();
        if (mv) {
            s.msg[ln + 1] = mine;
            s.cnt[ln + 1] = c;
        }
        if (ln == 0) {
            s.msg[k] = m;
            s.cnt[k] = 1;
            s.nmsg = (uint8_t)(n + 1);
        }
        w_wsync();
        return W_ON;
    }
    static __device__ void remove_at(WState& s, int k) {  // wbag_remove_at
        const int ln = (int)__lane_id();
        w_wsync();
        const int c = s.cnt[k], n = s.nmsg;
        if (c > 1) {
            w_wsync();
            if (ln == 0) s.cnt[k] = (uint8_t)(c - 1);
            w_wsync();
            return;
        }
        const bool mv = ln > k && ln < n;  // messages k+1 .. n-1 move down one slot
        WMsg mine;
        uint8_t cm = 0;
        if (mv) {
            mine = s.msg[ln];
            cm = s.cnt[ln];
        }
        w_wsync();
        if (mv) {
            s.msg[ln - 1] = mine;
            s.cnt[ln - 1] = cm;
        }
        if (ln == n - 1) {  // the freed last slot (also written by no mover: n - 1 > ln - 1)
            wmsg_zero(s.msg[n - 1]);
            s.cnt[n - 1] = 0;
        }
        if (ln == 0) s.nmsg = (uint8_t)(n - 1);
        w_wsync();
    }
};

// win_model with lane q checking message q's count.
__device__ __forceinline__ int w_in_model_wave(const WModel& M, const WState& t) {
    const int ln = (int)__lane_id();
    bool bad = ln < t.nmsg && t.cnt[ln] > M.max_dup;
    if (ln < M.S) bad = bad || t.ct[ln] > M.max_term || t.len[ln] > M.max_log;
    if (ln == 0) bad = bad || t.nmsg > M.max_msgs;
    return __ballot(bad) == 0;
}

// TypeOK (raft.tla:482-492, wtype_ok) with lane i checking server i and lane q
// message q.
__device__ __forceinline__ int w_type_ok_wave(const WModel& M, const WState& s) {
    const int ln = (int)__lane_id();
    bool bad = false;
    if (ln < M.S) {
        const int i = ln;
        bad = s.st[i] > LEADER || (s.vf[i] != NIL && s.vf[i] >= M.S) || ((s.vR[i] | s.vG[i]) >> M.S) != 0;
        for (int j = 0; j < M.S; ++j) bad = bad || s.ni[i][j] < 1;
        for (int x = 0; x < s.len[i]; ++x) bad = bad || s.log[i][x].value >= M.V;
    }
    if (ln < s.nmsg) {
        const WMsg& m = s.msg[ln];
        bad = bad || s.cnt[ln] < 1 || m.src >= M.S || m.dst >= M.S;
        for (int x = 0; x < m.n; ++x) bad = bad || m.e[x].value >= M.V;
    }
    return __ballot(bad) == 0;
}

// wcheck_invariants for the whole wave (every lane gets the result): TypeOK
// lane-parallel, the other named invariants on lane 0 in wcheck_invariants'
// order.
__device__ __forceinline__ int w_check_invariants_wave(const WModel& M, const WState& s) {
    if ((M.inv_mask & 1) && !w_type_ok_wave(M, s)) return 1;
    if (!(M.inv_mask & ~1)) return 0;
    WModel M2 = M;
    M2.inv_mask &= ~1;
    const int v = __lane_id() == 0 ? wcheck_invariants(M2, s) : 0;
    return __shfl(v, 0);
}

// Random behaviours (TLC -simulate): one thread per behaviour, from one of the
// n_init staged initial states, up to depth - 1 steps.  mode 0: uniform over
// the enabled successors within the bounds (rejection: an out-of-bounds draw
// is excluded and the draw repeated; uniform_draw); 1: uniform over every enabled successor,
// one beyond the bounds ends the behaviour (truncated); 2: TLC's draw
// (tlc_draw: random start, random prime stride, the first enabled action, a
// uniform successor of it); beyond the bounds it is truncated like mode 1.
__global__ __launch_bounds__(64) void k_wsimulate(const WModel M, const WState* inits, u64 n_init, u64 n_beh, int depth,
                                                 u64 seed, int mode, SimCounters* out, i64 rec_beh, WState* rec) {
    u64 steps = 0, trunc = 0, dead = 0;
    const int nl = M.L.off[10];
    const int o7 = M.L.off[7], o8 = M.L.off[8], o9 = M.L.off[9];
    for (u64 b = (u64)blockIdx.x * 64ull + threadIdx.x; b < n_beh; b += (u64)gridDim.x * 64ull) {
        if (rec_beh >= 0 && (i64)b != rec_beh) continue;
        u64 rs = mix64(seed ^ (b * 0xD1B54A32D192ED03ull));
        // two records used in turn (the successor becomes the current state by
        // swapping the roles, not by a 5-KB copy)
        WState buf[2];
        int cur = 0;
        wcopy_state(buf[0], inits[w_rand(rs) % n_init]);
        const bool record = (i64)b == rec_beh;
        if (record) wcopy_state(rec[0], buf[cur]);
        int v = wcheck_invariants(M, buf[cur]);
        if (v) atomicMin((unsigned long long*)&out->viol, (unsigned long long)((1ull << 44) | ((u64)(v - 1) << 40) | b));
        u64 excl[WLMASK] = {};  // mode 0: lanes whose successor left the bounds this step
        for (int dd = 2; dd <= depth && !v;) {
            u64 en[WLMASK] = {};
            for (int lane = 0; lane < nl; ++lane)
                if (wlane(M, buf[cur], lane, nullptr) != W_OFF) en[lane >> 6] |= 1ull << (lane & 63);
            const int pick = mode == 2 ? tlc_draw<WLMASK>(en, nl, o7, o8, o9, rs)  // TLC's draw
                                       : uniform_draw<WLMASK>(en, excl, rs);
            if (pick < 0) {
                u64 any = 0;
                for (int q = 0; q < WLMASK; ++q) any |= excl[q];
                if (any) ++trunc;  // mode 0: every enabled successor leaves the bounds
                else ++dead;
                break;
            }
            const int r = wlane(M, buf[cur], pick, &buf[cur ^ 1]);
            if (r != W_ON || !win_model(M, buf[cur ^ 1])) {
                if (mode == 0) {  // exclude it and draw again (a lane whose successor overflows too)
                    excl[pick >> 6] |= 1ull << (pick & 63);
                    continue;
                }
                ++trunc;
                break;
            }
            cur ^= 1;
            for (int q = 0; q < WLMASK; ++q) excl[q] = 0;
            ++steps;
            if (record) wcopy_state(rec[dd - 1], buf[cur]);
            v = wcheck_invariants(M, buf[cur]);
            if (v)
                atomicMin((unsigned long long*)&out->viol, (unsigned long long)(((u64)dd << 44) | ((u64)(v - 1) << 40) | b));
            ++dd;
        }
    }
    atomicAdd((unsigned long long*)&out->steps, (unsigned long long)steps);
    if (trunc) atomicAdd((unsigned long long*)&out->truncated, (unsigned long long)trunc);
    if (dead) atomicAdd((unsigned long long*)&out->deadlocked, (unsigned long long)dead);
}

// The same walks, one WAVE per behaviour (RMC_WSIM=1, the default): the two
// 5-KB records live in LDS instead of one lane's private memory, the 64 lanes
// evaluate the action guards in parallel (a ballot per 64 lanes of the lane
// table), copy the record together, apply the drawn action together (the
// scalar fields by every lane alike, the bag one message per lane: WaveBag)
// and check TypeOK and the CONSTRAINT one server / message per lane.  The
// draws are the thread kernel's (the same random stream per behaviour), so
// both give the same behaviours.
constexpr int WSIM_WAVES = 4;  // behaviours per 256-thread block (2 x 5,080 B of LDS each)
__global__ __launch_bounds__(64 * WSIM_WAVES) __attribute__((amdgpu_waves_per_eu(4))) void k_wsimulate_w(const WModel M, const WState* inits, u64 n_init,
                                                                u64 n_beh, int depth, u64 seed, int mode,
                                                                SimCounters* out, i64 rec_beh, WState* rec,
                                                                int inplace) {
    __shared__ WState s_buf[WSIM_WAVES][2];
    const int wv = (int)(threadIdx.x >> 6), ln = (int)(threadIdx.x & 63);
    u64 steps = 0, trunc = 0, dead = 0;  // lane 0's tallies
    const int nl = M.L.off[10];
    const int o7 = M.L.off[7], o8 = M.L.off[8], o9 = M.L.off[9];
    constexpr int NC = (WLANES_MAX + 63) / 64;  // 64-lane chunks of the lane table
    auto copy = [&](WState& d, const WState& s) {  // the whole wave, 8 bytes a lane at a time
        u64* x = reinterpret_cast<u64*>(&d);
        const u64* y = reinterpret_cast<const u64*>(&s);
        for (int k = ln; k < WWORDS; k += 64) x[k] = y[k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (u64 b = (u64)blockIdx.x * WSIM_WAVES + wv; b < n_beh; b += (u64)gridDim.x * WSIM_WAVES) {  // wave-uniform
        if (rec_beh >= 0 && (i64)b != rec_beh) continue;
        u64 rs = mix64(seed ^ (b * 0xD1B54A32D192ED03ull));  // every lane: the same stream
        int cur = 0;
        copy(s_buf[wv][0], inits[w_rand(rs) % n_init]);
        const bool record = (i64)b == rec_beh;
        if (record && ln == 0) wcopy_state(rec[0], s_buf[wv][0]);
        int v = w_check_invariants_wave(M, s_buf[wv][0]);
        if (v && ln == 0)
            atomicMin((unsigned long long*)&out->viol, (unsigned long long)((1ull << 44) | ((u64)(v - 1) << 40) | b));
        u64 excl[WLMASK] = {};  // mode 0: lanes whose successor left the bounds this step (uniform)
        for (int dd = 2; dd <= depth && !v;) {
            const WState& s = s_buf[wv][cur];
            // guards in parallel: en[c] bit l = lane 64 c + l enabled (wave-uniform masks)
            u64 en[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int lane = 64 * c + ln;
                const bool on = lane < nl && wlane(M, s, lane, nullptr) != W_OFF;
                en[c] = __ballot(on);
            }
            static_assert(NC == WLMASK, "one mask word per 64 lanes");
            const int pick = mode == 2 ? tlc_draw<NC>(en, nl, o7, o8, o9, rs)  // k_wsimulate's draws exactly
                                       : uniform_draw<NC>(en, excl, rs);
            if (pick < 0) {
                u64 any = 0;
                for (int q = 0; q < WLMASK; ++q) any |= excl[q];
                if (any) ++trunc;
                else ++dead;
                break;
            }
            // mode 0 may redraw from s: the successor goes to the other record.
            // Otherwise a failed draw ends the behaviour, so the successor is
            // written over s in place (wlane reads every field of s before it
            // writes it) and the 5-KB copy is skipped.
            const bool inp = inplace && mode != 0;
            WState& t = s_buf[wv][inp ? cur : cur ^ 1];
            if (!inp) copy(t, s);
            const int r = wlane<WaveBag>(M, s, pick, &t, true);  // every lane: the same r
            w_wsync();
            if (r != W_ON || !w_in_model_wave(M, t)) {
                if (mode == 0) {
                    excl[pick >> 6] |= 1ull << (pick & 63);
                    continue;
                }
                ++trunc;
                break;
            }
            if (!inp) cur ^= 1;
            for (int q = 0; q < WLMASK; ++q) excl[q] = 0;
            ++steps;
            if (record && ln == 0) wcopy_state(rec[dd - 1], t);
            v = w_check_invariants_wave(M, t);
            if (v && ln == 0)
                atomicMin((unsigned long long*)&out->viol, (unsigned long long)(((u64)dd << 44) | ((u64)(v - 1) << 40) | b));
            ++dd;
        }
    }
    if (ln == 0) {
        atomicAdd((unsigned long long*)&out->steps, (unsigned long long)steps);
        if (trunc) atomicAdd((unsigned long long*)&out->truncated, (unsigned long long)trunc);
        if (dead) atomicAdd((unsigned long long*)&out->deadlocked, (unsigned long long)dead);
    }
}

// ---- host launchers ---------------------------------------------------------------
static unsigned grid_for(u64 n, u64 threads, u64 maxg) {
    const u64 b = (n + threads - 1) / threads;
    return (unsigned)(b < maxg ? (b ? b : 1) : maxg);
}

hipError_t launch_wseed(const WModel& M, const WideBufs& B, const void* staged, u64 n, hipStream_t st) {
    if (!n) return hipSuccess;
    if (B.compact == 2)
        hipLaunchKernelGGL(k_wseed<WStateD>, dim3(grid_for(n, 256, 1024)), dim3(256), 0, st, M, B,
                           static_cast<const WStateD*>(staged), n);
    else if (B.compact)
        hipLaunchKernelGGL(k_wseed<WStateC>, dim3(grid_for(n, 256, 1024)), dim3(256), 0, st, M, B,
                           static_cast<const WStateC*>(staged), n);
    else
        hipLaunchKernelGGL(k_wseed<WState>, dim3(grid_for(n, 256, 1024)), dim3(256), 0, st, M, B,
                           static_cast<const WState*>(staged), n);
    return hipGetLastError();
}
hipError_t launch_wexpand(const WModel& M, const WideBufs& B, u64 lo, u64 hi, hipStream_t st) {
    if (hi <= lo) return hipSuccess;
    if (B.compact == 2)
        hipLaunchKernelGGL(k_wexpand<WStateD>, dim3(grid_for(hi - lo, 256, 4096)), dim3(256), 0, st, M, B, lo, hi);
    else if (B.compact)
        hipLaunchKernelGGL(k_wexpand<WStateC>, dim3(grid_for(hi - lo, 256, 4096)), dim3(256), 0, st, M, B, lo, hi);
    else
        hipLaunchKernelGGL(k_wexpand<WState>, dim3(grid_for(hi - lo, 256, 4096)), dim3(256), 0, st, M, B, lo, hi);
    return hipGetLastError();
}
hipError_t launch_wlist(const WModel& M, const WState* in, u64 n, WSucc* out, u64 cap, unsigned long long* count,
                        u64 salt, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_wlist, dim3(grid_for(n, 64, 1u << 20)), dim3(64), 0, st, M, in, n, out, cap, count, salt);
    return hipGetLastError();
}
hipError_t launch_wsimulate(const WModel& M, const WState* inits, u64 n_init, u64 n_beh, int depth, u64 seed, int mode,
                            SimCounters* out, i64 rec_beh, WState* rec, hipStream_t st) {
    static const int wave = [] {  // RMC_WSIM=0: one thread per behaviour (k_wsimulate, A/B)
        const char* e = getenv("RMC_WSIM");
        return e ? atoi(e) : 1;
    }();
    static const int inplace = [] {  // RMC_WSIM_INPLACE=0: every successor to the other record (A/B)
        const char* e = getenv("RMC_WSIM_INPLACE");
        return e ? atoi(e) : 1;
    }();
    if (wave)
        hipLaunchKernelGGL(k_wsimulate_w, dim3(grid_for(n_beh, WSIM_WAVES, 8192)), dim3(64 * WSIM_WAVES), 0, st, M,
                           inits, n_init, n_beh, depth, seed, mode, out, rec_beh, rec, inplace);
    else
        hipLaunchKernelGGL(k_wsimulate, dim3(grid_for(n_beh, 64, 16384)), dim3(64), 0, st, M, inits, n_init, n_beh,
                           depth, seed, mode, out, rec_beh, rec);
    return hipGetLastError();
}

}  // namespace wide
}  // namespace rmc
