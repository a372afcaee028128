/* ref_pin_time.c -- TEST INFRASTRUCTURE ONLY.  Linked into the reference's
 * unmodified libfm.cpp (oracle/Makefile _ref/libFM): libfm.cpp:124 seeds the
 * RNG with time(NULL) and ignores -seed, so this time() returns the value of
 * $LIBFM_PIN_TIME (default 1), which makes libFM's MCMC chains reproducible
 * and comparable with oracle/fmm_oracle.c at seed = that value. */
#include <stdlib.h>
#include <time.h>

time_t time(time_t *t) {
    const char *s = getenv("LIBFM_PIN_TIME");
    const time_t v = s ? (time_t)atol(s) : (time_t)1;
    if (t) *t = v;
    return v;
}
