// Host build of se3-icp_amd/csrc/pairmath.hpp (the per-pair solve and loop state machine
// that k_reduce_final runs on the GPU) for tests/test_pairmath.py: reads cases from
// stdin, writes results to stdout, one line per case.
//   U <15 moments> <n>        -> umeyama_from_moments: 16 values (row-major 4x4)
//   N <27 normal-eq values>   -> solve_normal_equations: 16 values
//   S <16 T> <kind> <est> <sw> <iter> <max_iter> <max_se3> <mse> <mse_switch> <sf> <K>
//     <mse_cur> <28 reduced values>
//                             -> pair_close_iteration then pair_open_iteration:
//                                iter pure sw done phase phase_start mse_cur rel + 16 T
#include <cstdio>
#include <iostream>
#include <string>

#include "pairmath.hpp"

using namespace se3icp;

static void print_m4(const M4& T) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) std::printf(" %.17g", T.m[i][j]);
}

int main() {
    std::string tag;
    while (std::cin >> tag) {
        if (tag == "U") {
            double s[15], n;
            for (double& x : s) std::cin >> x;
            std::cin >> n;
            print_m4(umeyama_from_moments(s, n));
        } else if (tag == "N") {
            double a[27];
            for (double& x : a) std::cin >> x;
            print_m4(solve_normal_equations(a));
        } else if (tag == "S") {
            PairState S{};
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) std::cin >> S.T.m[i][j];
            int est;
            std::cin >> S.kind >> est >> S.sw >> S.iter >> S.max_iter >> S.max_se3 >> S.mse >> S.mse_switch >> S.sf >>
                S.K >> S.mse_cur;
            double acc[28];
            for (double& x : acc) std::cin >> x;
            S.phase = PHASE_SE3;
            S.phase_start = 1;
            PairDev P{};
            pair_close_iteration(S, est, acc);
            pair_open_iteration(S, P);
            std::printf("%d %d %d %d %d %d %.17g %.17g", S.iter, S.pure, S.sw, S.done, P.phase, S.phase_start,
                        S.mse_cur, S.rel);
            print_m4(S.T);
        } else {
            return 2;
        }
        std::printf("\n");
    }
    return 0;
}
