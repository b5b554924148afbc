// Host check of the simulators' TLC draw (raft_wide.h tlc_draw): over random
// sets of enabled lanes of the wide lane table (S = 3 and 5), the frequency of
// every drawn lane over many draws equals the exact probability of the stated
// rule — a uniformly random start among Next's actions, a uniformly random
// prime stride from the table, the first action with a successor, then one of
// its enabled lanes uniformly — to within 6 standard deviations.  Also reports
// how far the rule is from "uniform over the enabled actions" (it is not that).
// Build: g++ -O2 -std=c++17 -I raft.tla_amd/csrc tlc_draw_check.cpp
// Run:   ./a.out <masks> <draws per mask> <seed>   (prints "ok ..." or the first failure)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "raft_wide.h"

using namespace rmc;
using namespace rmc::wide;

int main(int argc, char** argv) {
    const int masks = argc > 1 ? atoi(argv[1]) : 40;
    const int draws = argc > 2 ? atoi(argv[2]) : 200000;
    u64 x = argc > 3 ? strtoull(argv[3], nullptr, 10) : 1;
    constexpr int NC = (WLANES_MAX + 63) / 64;
    const u32 primes[8] = {89, 97, 101, 103, 107, 109, 113, 127};
    double worst = 0, nonuni = 0;
    for (int S : {3, 5}) {
        WLanes L;
        L.init(S);
        const int nl = L.off[10], o7 = L.off[7], o8 = L.off[8], o9 = L.off[9], nact = o7 + 3;
        for (int t = 0; t < masks; ++t) {
            u64 en[NC] = {};
            const u64 dens = w_rand(x) % 4;  // some masks sparse, some dense
            const int nmsg = (int)(w_rand(x) % 12);
            for (int lane = 0; lane < nl; ++lane) {
                if (lane >= o7 && (lane - (lane < o8 ? o7 : lane < o9 ? o8 : o9)) >= nmsg) continue;
                if (w_rand(x) % 4 <= dens) en[lane >> 6] |= 1ull << (lane & 63);
            }
            auto on = [&](int l) { return ((en[l >> 6] >> (l & 63)) & 1ull) != 0; };
            auto fam = [&](int f, int* lo, int* hi) {
                *lo = f == 0 ? o7 : f == 1 ? o8 : o9;
                *hi = f == 0 ? o8 : f == 1 ? o9 : nl;
            };
            int n_on_act = 0;
            for (int a = 0; a < nact; ++a) {
                bool any = false;
                if (a < o7) {
                    any = on(a);
                } else {
                    int lo, hi;
                    fam(a - o7, &lo, &hi);
                    for (int l = lo; l < hi; ++l) any |= on(l);
                }
                n_on_act += any;
            }
            if (!n_on_act) continue;
            // exact probability of each lane under the rule
            std::vector<double> p(nl, 0.0);
            for (int st = 0; st < nact; ++st)
                for (u32 pr : primes)
                    for (int i = 0; i < nact; ++i) {
                        const int a = (int)((st + (u32)i * pr) % (u32)nact);
                        if (a < o7) {
                            if (on(a)) {
                                p[a] += 1.0 / (nact * 8.0);
                                break;
                            }
                            continue;
                        }
                        int lo, hi, cnt = 0;
                        fam(a - o7, &lo, &hi);
                        for (int l = lo; l < hi; ++l) cnt += on(l);
                        if (!cnt) continue;
                        for (int l = lo; l < hi; ++l)
                            if (on(l)) p[l] += 1.0 / (nact * 8.0) / cnt;
                        break;
                    }
            std::vector<int> h(nl, 0);
            u64 rs = w_rand(x);
            for (int d = 0; d < draws; ++d) {
                const int l = tlc_draw<NC>(en, nl, o7, o8, o9, rs);
                if (l < 0 || !on(l)) {
                    printf("FAIL S=%d mask %d: drew lane %d, not enabled\n", S, t, l);
                    return 1;
                }
                ++h[l];
            }
            for (int l = 0; l < nl; ++l) {
                if (p[l] == 0) {
                    if (h[l]) {
                        printf("FAIL S=%d mask %d: lane %d drawn, probability 0\n", S, t, l);
                        return 1;
                    }
                    continue;
                }
                const double e = p[l] * draws, sd = std::sqrt(e * (1 - p[l]));
                const double z = std::fabs(h[l] - e) / sd;
                if (z > 6.0) {
                    printf("FAIL S=%d mask %d lane %d: %d draws, expected %.1f (z %.1f)\n", S, t, l, h[l], e, z);
                    return 1;
                }
                worst = std::max(worst, z);
            }
            for (int a = 0; a < o7; ++a)  // distance from "uniform over the enabled actions"
                if (on(a)) nonuni = std::max(nonuni, std::fabs(p[a] - 1.0 / n_on_act));
        }
    }
    printf("ok worst z %.2f; max |P(action) - 1/(enabled actions)| %.4f\n", worst, nonuni);
    return 0;
}
