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
 * Every exchange is checked: before it arrives, a rank publishes (exchange number, bytes) in
 * its own header slot (two alternating slot sets, like the areas), and after the wait every
 * rank compares all slots with its own -- ranks whose control flow diverged (a different
 * batch, a different size) fail with an error instead of mixing results.  The slot also
 * carries a flag word; every rank gets the OR of all ranks' flags (fh_shm_allgather_flags:
 * collective decisions such as the SIGINT dump, scan-chromosome.c:557-569).
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
#define SHM_MAX_RANKS 64

typedef struct {                     /* one rank's view of one exchange */
  _Atomic unsigned long long seq;    /* exchange number (1-based) */
  unsigned long long bytes;          /* n * item */
  unsigned int flags;
  unsigned int pad;
} shm_slot_t;

typedef struct {
  _Atomic unsigned long long arrive; /* arrivals over all exchanges */
  _Atomic unsigned int attached;
  _Atomic unsigned int magic;
  unsigned int world;
  unsigned int pad;
  unsigned long long cap;            /* bytes per area */
  char fill[128 - 32];
  shm_slot_t slot[2][SHM_MAX_RANKS]; /* by exchange parity, as the areas */
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
  fh_shm_t *m;
  const size_t bytes = sizeof(shm_hdr_t) + 2 * cap;
  int fd = -1;
  const double t0 = fh_now();
  if (world < 1 || world > SHM_MAX_RANKS || rank < 0 || rank >= world) {
    logmsg(MSG_ERROR, "fscl_amd: shm exchange: rank %d of %d (at most %d ranks)", rank, world, SHM_MAX_RANKS);
    return NULL;
  }
  m = fh_calloc(1, sizeof *m, "shm");
  m->rank = rank; m->world = world; m->map_bytes = bytes;
  if (rank == 0) {
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) {
      if (errno == EEXIST)
        logmsg(MSG_ERROR, "fscl_amd: shm segment %s already exists: another job of the same name is running, or "
                          "an earlier one died before all its ranks attached (remove /dev/shm%s, or set "
                          "FSCL_AMD_SHM_NAME)", name, name);
      else
        logmsg(MSG_ERROR, "fscl_amd: shm_open(%s): %s", name, strerror(errno));
      free(m);
      return NULL;
    }
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

/* all-gather of n items of `item` bytes: this rank owns [lo, hi) of buf.  *flags (may be
   NULL) is this rank's flag word on entry and the OR over all ranks on return.  Every rank
   must make the same exchanges with the same n * item: checked, a mismatch is an error. */
int fh_shm_allgather_flags(fh_shm_t *m, void *buf, size_t item, int n, int lo, int hi, unsigned *flags) {
  const int par = (int)(m->seq & 1);
  char *a = m->area[par];
  const unsigned long long want = (unsigned long long)n * item, next = m->seq + 1;
  unsigned any = 0;
  int r;
  if (want > m->h->cap) {
    logmsg(MSG_ERROR, "fscl_amd: rank exchange of %llu bytes above the segment's %llu (FSCL_AMD_SHM_MB)",
           want, m->h->cap);
    return -1;
  }
  if (hi > lo) memcpy(a + (size_t)lo * item, (char *)buf + (size_t)lo * item, (size_t)(hi - lo) * item);
  {
    shm_slot_t *me = &m->h->slot[par][m->rank];
    me->bytes = want;
    me->flags = flags ? *flags : 0u;
    atomic_store_explicit(&me->seq, next, memory_order_release);
  }
  atomic_fetch_add_explicit(&m->h->arrive, 1ull, memory_order_acq_rel);
  m->seq = next;
  if (wait_ge_ull(&m->h->arrive, m->seq * (unsigned long long)m->world) != 0) {
    logmsg(MSG_ERROR, "fscl_amd: rank exchange timed out (a rank stopped)");
    return -1;
  }
  for (r = 0; r < m->world; r++) {
    shm_slot_t *o = &m->h->slot[par][r];
    const unsigned long long sq = atomic_load_explicit(&o->seq, memory_order_acquire);
    if (sq != next || o->bytes != want) {
      logmsg(MSG_ERROR, "fscl_amd: rank exchange mismatch: rank %d is at exchange %llu with %llu bytes, rank %d at "
                        "%llu with %llu (the ranks' control flow diverged)", r, sq, o->bytes, m->rank, next, want);
      return -1;
    }
    any |= o->flags;
  }
  if (flags) *flags = any;
  if (n > 0) memcpy(buf, a, (size_t)want);
  return 0;
}

int fh_shm_allgather(fh_shm_t *m, void *buf, size_t item, int n, int lo, int hi) {
  return fh_shm_allgather_flags(m, buf, item, n, lo, hi, NULL);
}

/* a barrier: an all-gather of nothing */
int fh_shm_barrier(fh_shm_t *m) {
  char dummy = 0;
  return fh_shm_allgather_flags(m, &dummy, 1, 0, 0, 0, NULL);
}
