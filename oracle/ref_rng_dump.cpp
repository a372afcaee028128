// ref_rng_dump.cpp -- TEST INFRASTRUCTURE ONLY.  Dumps the reference's own RNG
// (src/util/random.h, included from where it lies) for golden vectors:
//   ref_rng_dump SEED N   ->  N lines "rand uniform gaussian" then gammas.
#include <cstdio>
#include <cstdlib>
#include "random.h"
int main(int argc, char** argv) {
    unsigned seed = argc > 1 ? (unsigned)strtoul(argv[1], 0, 10) : 1;
    int n = argc > 2 ? atoi(argv[2]) : 1000;
    srand(seed);
    for (int i = 0; i < n; i++) printf("rand %d\n", rand());
    srand(seed);
    for (int i = 0; i < n; i++) printf("gauss %.17g\n", ran_gaussian());
    const double shapes[] = {1.0 + 90570 / 2.0, 1.0 + 0.5 * 944, 0.7, 2.5, 1.0};
    for (double a : shapes) {
        srand(seed);
        for (int i = 0; i < n / 10; i++) printf("gamma %.17g %.17g\n", a, ran_gamma(a));
    }
    return 0;
}
