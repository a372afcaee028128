// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
// Linked beside the UNMODIFIED reference sampler sources (compiled where they
// lie under /root/reference) to make their output usable as golden vectors:
//  * seeds glibc rand() from $SBMF_REF_SEED before main() runs (the reference
//    samplers never call srand(), so without this the seed is glibc's 1);
//  * prints doubles with 17 significant digits instead of cout's default 6.
// It adds no code to the sampler and replaces nothing the image lacks.
#include <cstdlib>
#include <iostream>
namespace {
struct RefHarness {
    RefHarness() {
        if (const char* s = std::getenv("SBMF_REF_SEED")) std::srand((unsigned)std::strtoul(s, nullptr, 10));
        std::cout.precision(17);
    }
} ref_harness_instance;
}  // namespace
