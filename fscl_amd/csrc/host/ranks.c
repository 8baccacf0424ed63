/* ranks.c -- the exchange step of multi-process parity mode (one process per GPU on one
 * node): after every search batch each rank holds the results of its own share of the
 * batch's cells, and every rank needs all of them (each rank runs the reference's pruning,
 * scan-chromosome.c:488-502, on the whole point set).  The results live in host memory
 * (the pruning is host code), and all ranks share one node, so the exchange is an
 * all-gather through a POSIX shared-memory segment: a rank writes its contiguous share,
 * arrives at a counter, waits for the others and reads the whole batch -- a few
 * microseconds, with no device round trip.  Two alternating areas make one arrival per
 * exchange enough: a rank writes area k%2 only after every rank has arrived at exchange
 * k-1, i.e. has finished reading area (k-2)%2.
 *
 * The segment is created by rank 0 under a name unique to the job (O_EXCL), mapped by every
 * rank, and unlinked by rank 0 once all have attached, so nothing is left in /dev/shm even
 * if a rank dies later.  Every wait has a time limit (FSCL_AMD_RANK_TIMEOUT seconds,
 * default 600): a rank that never arrives ends the job with a fatal error, not a hang.
 */
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "fscl_host.h"

#define SHM_MAGIC 0x6673636cu /* "fscl" */

typedef struct {
  _Atomic unsigned long long arrive; /* arrivals over all exchanges */
  _Atomic unsigned int attached;
  _Atomic unsigned int magic;
  unsigned int world;
  unsigned int pad;
  unsigned long long cap;            /* bytes per area */
  char fill[128 - 32];
} shm_hdr_t;

struct fh_shm {
  shm_hdr_t *h;
  char *area[2];
  size_t map_bytes;
  unsigned long long seq;  /* exchanges done by this rank */
  int rank, world;
};

static double timeout_s(void) {
  const char *e = getenv("FSCL_AMD_RANK_TIMEOUT");
  return e && atof(e) > 0 ? atof(e) : 600.0;
}

/* spin (then yield) until *v >= target, or fail after the time limit */
static int wait_ge_ull(_Atomic unsigned long long *v, unsigned long long target) {
  const double t0 = fh_now(), lim = timeout_s();
  unsigned long spins = 0;
  while (atomic_load_explicit(v, memory_order_acquire) < target) {
    if (++spins > 4096) {
      sched_yield();
      if ((spins & 1023) == 0 && fh_now() - t0 > lim) return -1;
    }
  }
  return 0;
}

static int wait_ge_u(_Atomic unsigned int *v, unsigned int target) {
  const double t0 = fh_now(), lim = timeout_s();
  while (atomic_load_explicit(v, memory_order_acquire) < target) {
    usleep(100);
    if (fh_now() - t0 > lim) return -1;
  }
  return 0;
}

fh_shm_t *fh_shm_open(int rank, int world, const char *name, size_t cap) {
  fh_shm_t *m = fh_calloc(1, sizeof *m, "shm");
  const size_t bytes = sizeof(shm_hdr_t) + 2 * cap;
  int fd = -1;
  const double t0 = fh_now();
  m->rank = rank; m->world = world; m->map_bytes = bytes;
  if (rank == 0) {
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) { logmsg(MSG_ERROR, "fscl_amd: shm_open(%s): %s", name, strerror(errno)); free(m); return NULL; }
    if (ftruncate(fd, (off_t)bytes) != 0) {
      logmsg(MSG_ERROR, "fscl_amd: ftruncate(%s): %s", name, strerror(errno));
      close(fd); shm_unlink(name); free(m); return NULL;
    }
  } else {
    for (;;) {  /* rank 0 creates it */
      struct stat sb;
      fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0 && fstat(fd, &sb) == 0 && (size_t)sb.st_size >= bytes) break;
      if (fd >= 0) close(fd);
      if (fh_now() - t0 > timeout_s()) { logmsg(MSG_ERROR, "fscl_amd: shm %s never appeared", name); free(m); return NULL; }
      usleep(1000);
    }
  }
  m->h = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m->h == MAP_FAILED) { logmsg(MSG_ERROR, "fscl_amd: mmap: %s", strerror(errno)); free(m); return NULL; }
  m->area[0] = (char *)m->h + sizeof(shm_hdr_t);
  m->area[1] = m->area[0] + cap;
  if (rank == 0) {
    m->h->world = (unsigned)world;
    m->h->cap = cap;
    atomic_store_explicit(&m->h->magic, SHM_MAGIC, memory_order_release);
  } else if (wait_ge_u(&m->h->magic, SHM_MAGIC) != 0 || m->h->world != (unsigned)world || m->h->cap != cap) {
    logmsg(MSG_ERROR, "fscl_amd: shm %s: rank set mismatch", name);
    munmap(m->h, bytes); free(m); return NULL;
  }
  atomic_fetch_add_explicit(&m->h->attached, 1u, memory_order_acq_rel);
  if (wait_ge_u(&m->h->attached, (unsigned)world) != 0) {
    logmsg(MSG_ERROR, "fscl_amd: shm %s: not every rank attached", name);
    munmap(m->h, bytes); free(m); return NULL;
  }
  if (rank == 0) shm_unlink(name);  /* every rank has it mapped */
  return m;
}

void fh_shm_close(fh_shm_t *m) {
  if (!m) return;
  munmap(m->h, m->map_bytes);
  free(m);
}

/* all-gather of n items of `item` bytes: this rank owns [lo, hi) of buf */
int fh_shm_allgather(fh_shm_t *m, void *buf, size_t item, int n, int lo, int hi) {
  char *a = m->area[m->seq & 1];
  if ((size_t)n * item > m->h->cap) {
    logmsg(MSG_ERROR, "fscl_amd: rank exchange of %zu bytes above the segment's %llu (FSCL_AMD_SHM_MB)",
           (size_t)n * item, m->h->cap);
    return -1;
  }
  if (hi > lo) memcpy(a + (size_t)lo * item, (char *)buf + (size_t)lo * item, (size_t)(hi - lo) * item);
  atomic_fetch_add_explicit(&m->h->arrive, 1ull, memory_order_acq_rel);
  m->seq++;
  if (wait_ge_ull(&m->h->arrive, m->seq * (unsigned long long)m->world) != 0) {
    logmsg(MSG_ERROR, "fscl_amd: rank exchange timed out (a rank stopped)");
    return -1;
  }
  memcpy(buf, a, (size_t)n * item);
  return 0;
}

/* a barrier: an all-gather of nothing */
int fh_shm_barrier(fh_shm_t *m) {
  char dummy = 0;
  return fh_shm_allgather(m, &dummy, 1, 0, 0, 0);
}
