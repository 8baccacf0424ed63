/* util.c -- allocation, clock, logging (logmsg.c:20-52), rand stream. */
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "fscl_host.h"

void *fh_malloc(size_t n, const char *where) {
  void *p = malloc(n ? n : 1);
  if (!p) { fprintf(stderr, "Failed allocating memory at %s (%1.1f Mb)\n", where, n / 1e6); abort(); }
  return p;
}
void *fh_calloc(size_t n, size_t m, const char *where) {
  void *p = calloc(n ? n : 1, m ? m : 1);
  if (!p) { fprintf(stderr, "Failed allocating memory at %s (%1.1f Mb)\n", where, n * (double)m / 1e6); abort(); }
  return p;
}
void *fh_realloc(void *p, size_t n, const char *where) {
  void *q = realloc(p, n ? n : 1);
  if (!q) { fprintf(stderr, "Failed allocating memory at %s (%1.1f Mb)\n", where, n / 1e6); abort(); }
  return q;
}
double fh_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* ---- logging: same levels and formats as logmsg.c ---- */
static int g_verbosity = MSG_STATUS;
static pthread_mutex_t g_log_lock = PTHREAD_MUTEX_INITIALIZER;

void configure_logmsg(int level) { g_verbosity = level; }

void logmsg(int priority, volatile char *s, ...) {
  va_list ap;
  char buf[4096];
  pthread_mutex_lock(&g_log_lock);
  if (priority <= g_verbosity) {
    va_start(ap, s);
    vsnprintf(buf, sizeof buf, (const char *)s, ap);
    va_end(ap);
    fprintf(stderr, "%s\n", buf);
  }
  pthread_mutex_unlock(&g_log_lock);
  if (priority == MSG_FATAL) exit(1);
}

void cr_logmsg(int priority, volatile char *s, ...) {
  va_list ap;
  char buf[4096];
  pthread_mutex_lock(&g_log_lock);
  if (priority <= g_verbosity) {
    va_start(ap, s);
    vsnprintf(buf, sizeof buf, (const char *)s, ap);
    va_end(ap);
    fprintf(stderr, "\33[2K\r%-79.79s", buf);
  }
  pthread_mutex_unlock(&g_log_lock);
  if (priority == MSG_FATAL) exit(1);
}

/* ---- glibc TYPE_3 additive-feedback generator (stdlib/random_r.c) ---- */
void fh_srand(fh_rand_t *g, unsigned seed) {
  int32_t word;
  int i;
  if (seed == 0) seed = 1;
  g->r[0] = word = (int32_t)seed;
  for (i = 1; i < 31; i++) {
    /* r[i] = 16807 * r[i-1] mod (2^31 - 1), Schrage's method */
    long hi = word / 127773, lo = word % 127773;
    word = (int32_t)(16807 * lo - 2836 * hi);
    if (word < 0) word += 2147483647;
    g->r[i] = word;
  }
  g->f = 3;
  g->b = 0;
  for (i = 0; i < 310; i++) fh_rand(g);
}

int fh_rand(fh_rand_t *g) {
  uint32_t v = (uint32_t)g->r[g->f] + (uint32_t)g->r[g->b];
  g->r[g->f] = (int32_t)v;
  if (++g->f == 31) g->f = 0;
  if (++g->b == 31) g->b = 0;
  return (int)(v >> 1);
}
