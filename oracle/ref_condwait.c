/* ref_condwait.c -- TEST INFRASTRUCTURE ONLY (oracle/_ref harness, own code).
 *
 * Linked into oracle/_ref/ref_driver with -Wl,--wrap=pthread_cond_wait so every
 * condition wait in the reference becomes a bounded (1 ms) timed wait.  POSIX
 * already allows spurious wake-ups and every reference wait sits in a predicate
 * loop (e.g. util/bgzf_output_stream.cpp:258-267), so this changes timing only.
 * It removes the reference's lost-wake-up deadlock in the BGZF writer (SURVEY Q13:
 * notify at util/bgzf_output_stream.cpp:54-56 can precede the wait at :266).
 */
#include <pthread.h>
#include <time.h>
#include <errno.h>

int __real_pthread_cond_wait(pthread_cond_t *c, pthread_mutex_t *m);

int __wrap_pthread_cond_wait(pthread_cond_t *c, pthread_mutex_t *m) {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    ts.tv_nsec += 1000000;
    if (ts.tv_nsec >= 1000000000) { ts.tv_sec += 1; ts.tv_nsec -= 1000000000; }
    int rc = pthread_cond_timedwait(c, m, &ts);
    return rc == ETIMEDOUT ? 0 : rc;
}
