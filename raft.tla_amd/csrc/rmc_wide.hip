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
__device__ __forceinline__ void w_store(const WModel& M, const WideBufs& B, u64 ni, const WState& t, u64 parent,
                                        int lane) {
    wcopy_state(B.store[ni], t);
    B.parent[ni] = parent;
    B.act[ni] = (uint8_t)lane;
    const int v = wcheck_invariants(M, t);
    if (v) atomicMin((unsigned long long*)&B.ctr->viol, (unsigned long long)((ni << 4) | (u64)(v - 1)));
}

// Init (raft.tla:125-129) or SmokeInit's states: n staged records.
__global__ __launch_bounds__(256) void k_wseed(const WModel M, const WideBufs B, const WState* staged, u64 n) {
    for (u64 t = (u64)blockIdx.x * 256ull + threadIdx.x; t < n; t += (u64)gridDim.x * 256ull) {
        if (!w_insert(B.table, B.tmask, wfp(staged[t], B.salt), &B.ctr->table_full)) continue;
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
// (Counters.overflow bits 8-11, the field).
__global__ __launch_bounds__(256) void k_wexpand(const WModel M, const WideBufs B, u64 lo, u64 hi) {
    u64 gen = 0, probes = 0;
    u32 bad = 0;
    const int nl = M.L.off[10];
    for (u64 i = lo + (u64)blockIdx.x * 256ull + threadIdx.x; i < hi; i += (u64)gridDim.x * 256ull) {
        WState s, t;
        wcopy_state(s, B.store[i]);
        u32 g = 0;
        for (int lane = 0; lane < nl; ++lane) {
            const int r = wlane(M, s, lane, &t);
            if (r == W_OFF) continue;
            ++g;
            if (r != W_ON) {  // beyond the layout: an error for a field no CONSTRAINT bounds,
                bad |= (u32)(woverflow_bits(r) & M.unbounded);  // else beyond its bound (filtered)
                continue;
            }
            if (!win_model(M, t)) continue;
            ++probes;
            if (!w_insert(B.table, B.tmask, wfp(t, B.salt), &B.ctr->table_full)) continue;
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
        w.fp = inm ? wfp(t, salt).k : 0ull;
        if (inm) wcopy_state(w.state, t);
        else wzero(&w.state, (int)sizeof(WState));
    }
}


// Random behaviours (TLC -simulate): one thread per behaviour, from one of the
// n_init staged initial states, up to depth - 1 steps.  mode 0: uniform over
// the enabled successors within the bounds (rejection: an out-of-bounds draw
// is excluded and the draw repeated); 1: uniform over every enabled successor,
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
            int pick = -1;
            if (mode == 2) {  // TLC's draw
                constexpr int NCL = (WLANES_MAX + 63) / 64;
                u64 en[NCL] = {};
                for (int lane = 0; lane < nl; ++lane)
                    if (wlane(M, buf[cur], lane, nullptr) != W_OFF) en[lane >> 6] |= 1ull << (lane & 63);
                pick = tlc_draw<NCL>(en, nl, o7, o8, o9, rs);
            } else {
                u32 cnt = 0;
                for (int lane = 0; lane < nl; ++lane) {  // reservoir: uniform over the enabled lanes
                    if ((excl[lane >> 6] >> (lane & 63)) & 1ull) continue;
                    if (wlane(M, buf[cur], lane, nullptr) == W_OFF) continue;
                    ++cnt;
                    if (w_rand(rs) % cnt == 0) pick = lane;
                }
            }
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
// table), copy the record together, and lane 0 applies the drawn action and
// checks the invariants.  The draws are the thread kernel's (the same random
// stream per behaviour), so both give the same behaviours.
constexpr int WSIM_WAVES = 4;  // behaviours per 256-thread block (2 x 5,080 B of LDS each)
__global__ __launch_bounds__(64 * WSIM_WAVES) void k_wsimulate_w(const WModel M, const WState* inits, u64 n_init,
                                                                u64 n_beh, int depth, u64 seed, int mode,
                                                                SimCounters* out, i64 rec_beh, WState* rec) {
    __shared__ WState s_buf[WSIM_WAVES][2];
    __shared__ int s_res[WSIM_WAVES];
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
        int v = ln == 0 ? wcheck_invariants(M, s_buf[wv][0]) : 0;
        v = __shfl(v, 0);
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
            int pick = -1;
            if (mode == 2) {  // TLC's draw, exactly as k_wsimulate
                pick = tlc_draw<NC>(en, nl, o7, o8, o9, rs);
            } else {  // reservoir over the enabled lanes in lane order (k_wsimulate's draws)
                u32 cnt = 0;
                for (int c = 0; c < NC; ++c)
                    for (u64 mm = en[c]; mm; mm &= mm - 1) {
                        const int lane = 64 * c + __builtin_ctzll(mm);
                        if ((excl[lane >> 6] >> (lane & 63)) & 1ull) continue;
                        ++cnt;
                        if (w_rand(rs) % cnt == 0) pick = lane;
                    }
            }
            if (pick < 0) {
                u64 any = 0;
                for (int q = 0; q < WLMASK; ++q) any |= excl[q];
                if (any) ++trunc;
                else ++dead;
                break;
            }
            WState& t = s_buf[wv][cur ^ 1];
            copy(t, s);
            if (ln == 0) {
                const int r = wlane(M, s, pick, &t, true);
                s_res[wv] = (r != W_ON || !win_model(M, t)) ? 1 : 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (s_res[wv]) {
                if (mode == 0) {
                    excl[pick >> 6] |= 1ull << (pick & 63);
                    continue;
                }
                ++trunc;
                break;
            }
            cur ^= 1;
            for (int q = 0; q < WLMASK; ++q) excl[q] = 0;
            ++steps;
            if (record && ln == 0) wcopy_state(rec[dd - 1], t);
            v = ln == 0 ? wcheck_invariants(M, t) : 0;
            v = __shfl(v, 0);
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

hipError_t launch_wseed(const WModel& M, const WideBufs& B, const WState* staged, u64 n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_wseed, dim3(grid_for(n, 256, 1024)), dim3(256), 0, st, M, B, staged, n);
    return hipGetLastError();
}
hipError_t launch_wexpand(const WModel& M, const WideBufs& B, u64 lo, u64 hi, hipStream_t st) {
    if (hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(k_wexpand, dim3(grid_for(hi - lo, 256, 4096)), dim3(256), 0, st, M, B, lo, hi);
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
    if (wave)
        hipLaunchKernelGGL(k_wsimulate_w, dim3(grid_for(n_beh, WSIM_WAVES, 8192)), dim3(64 * WSIM_WAVES), 0, st, M,
                           inits, n_init, n_beh, depth, seed, mode, out, rec_beh, rec);
    else
        hipLaunchKernelGGL(k_wsimulate, dim3(grid_for(n_beh, 64, 16384)), dim3(64), 0, st, M, inits, n_init, n_beh,
                           depth, seed, mode, out, rec_beh, rec);
    return hipGetLastError();
}

}  // namespace wide
}  // namespace rmc
