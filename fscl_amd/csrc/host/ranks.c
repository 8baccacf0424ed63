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
#include <signal.h>
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
  unsigned int creator;              /* rank 0's pid (a segment whose creator is gone is stale) */
  unsigned long long cap;            /* bytes per area */
  unsigned long long creator_ns;     /* the inode of rank 0's pid namespace: the pid means something only there */
  char fill[128 - 40];
  shm_slot_t slot[2][SHM_MAX_RANKS]; /* by exchange parity, as the areas */
} shm_hdr_t;

struct fh_shm {
  shm_hdr_t *h;
  char *area[2];
  size_t map_bytes;
  unsigned long long seq;  /* exchanges done by this rank */
  int rank, world;
  char name[200];          /* the segment's name: the permutation pools' names derive from it */
  unsigned n_pools;        /* pools opened so far (the same count on every rank: collective) */
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

/* this process's pid namespace (the inode of /proc/self/ns/pid; 0 if unknown) */
static unsigned long long pid_ns(void) {
  struct stat sb;
  return stat("/proc/self/ns/pid", &sb) == 0 ? (unsigned long long)sb.st_ino : 0ull;
}

/* 1 iff the segment's creator is provably gone: its pid is unknown to kill() AND it lives in our pid
   namespace.  Ranks in separate containers may share /dev/shm but not pids: a creator
   in another (or an unknown) namespace counts as alive. */
static int creator_dead(unsigned pid, unsigned long long ns) {
  const unsigned long long mine = pid_ns();
  if (!pid || !ns || !mine || ns != mine) return 0;
  return kill((pid_t)pid, 0) != 0 && errno == ESRCH;
}

/* A segment left by a launch that died before all its ranks attached (rank 0 unlinks the name
   only then): its creator is gone (creator_dead), or it was never initialised and is older than a
   minute.  Returns 1 for such a segment (the CLI's default name repeats across launches). */
static int shm_stale(const char *name) {
  struct stat sb;
  int stale = 0, fd = shm_open(name, O_RDONLY, 0600);
  if (fd < 0) return 0;
  if (fstat(fd, &sb) == 0) {
    if ((size_t)sb.st_size < sizeof(shm_hdr_t)) stale = time(NULL) - sb.st_ctime > 60;
    else {
      shm_hdr_t *h = mmap(NULL, sizeof(shm_hdr_t), PROT_READ, MAP_SHARED, fd, 0);
      if (h != MAP_FAILED) {
        const unsigned pid = h->creator;
        if (pid) stale = creator_dead(pid, h->creator_ns);
        else stale = time(NULL) - sb.st_ctime > 60;
        munmap(h, sizeof(shm_hdr_t));
      }
    }
  }
  close(fd);
  return stale;
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
  snprintf(m->name, sizeof m->name, "%s", name);
  if (rank == 0) {
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 && errno == EEXIST && shm_stale(name)) {
      logmsg(MSG_WARN, "fscl_amd: removing the stale shm segment %s (its launch died before every rank attached)\n",
             name);
      shm_unlink(name);
      fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    }
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
    for (;;) {  /* rank 0 creates it (a stale one left by a dead launch is skipped: rank 0 replaces it) */
      struct stat sb;
      fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0 && fstat(fd, &sb) == 0 && (size_t)sb.st_size >= bytes) {
        shm_hdr_t *h = mmap(NULL, sizeof(shm_hdr_t), PROT_READ, MAP_SHARED, fd, 0);
        int ok = 0;
        if (h != MAP_FAILED) {
          const int init = atomic_load_explicit(&h->magic, memory_order_acquire) == SHM_MAGIC;
          ok = init && h->creator && !creator_dead(h->creator, h->creator_ns);
          munmap(h, sizeof(shm_hdr_t));
        }
        if (ok) break;
      }
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
    m->h->creator = (unsigned)getpid();
    m->h->creator_ns = pid_ns();
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

int fh_shm_rank(const fh_shm_t *m) { return m->rank; }
int fh_shm_world(const fh_shm_t *m) { return m->world; }

/* ------------------------------------------------------------------ permutation pool
   One node leader (rank 0) builds each trial's block permutation once (scan-chromosome.c:
   441-456: the serial permutation at the trial barrier), with speculation over the whole
   node's spare CPUs, straight into buffers of a second shared-memory segment that every rank
   maps (and page-locks, so that its devices' scatter kernels read the rows from it directly).
   Per trial the leader publishes (rows offset, null-sums offset, rand() state after the
   permutation, negative-j count) in a ring; every other rank takes the publications in order,
   continues the rand() stream from the published state (the prune draws that follow are the
   same on every rank: same results, same order) and uploads the leader's rows.  A buffer is
   reused only after every rank has released the row slot that read it (per-rank release
   counters), and a ring entry only after every rank has taken it. */
#define POOL_RING 32
#define POOL_HDR (64u << 10)

typedef struct {
  unsigned long long seq;          /* 1-based publication number */
  unsigned long long rows_off, nul_off, negj;
  fh_rand_t end;                   /* the stream after this permutation */
} pool_pub_t;

typedef struct {
  _Atomic unsigned long long pub;                 /* publications so far */
  _Atomic unsigned long long cons[SHM_MAX_RANKS]; /* publications taken, per rank */
  _Atomic unsigned long long rel[SHM_MAX_RANKS];  /* row-slot releases, per rank */
  unsigned long long data_bytes;
  pool_pub_t ring[POOL_RING];
} pool_hdr_t;

_Static_assert(sizeof(pool_hdr_t) <= POOL_HDR, "pool header");

struct fh_pool {
  fh_shm_t *m;
  pool_hdr_t *h;
  char *data;
  size_t map_bytes, data_bytes;
  unsigned long long n_pub, n_take, n_rel;  /* this rank's counts */
};

/* collective (every rank of m, in the same order of calls): rank 0 creates a segment of
   data_bytes (the others' argument is ignored: they map what rank 0 made).  Returns NULL on
   every rank when rank 0 cannot reserve the memory (a small /dev/shm: the pages are allocated
   up front, so a short tmpfs fails here instead of faulting later) */
fh_pool_t *fh_pool_open(fh_shm_t *m, size_t data_bytes) {
  char name[256], dummy = 0;
  fh_pool_t *p = fh_calloc(1, sizeof *p, "pool");
  int fd = -1, err = 0;
  unsigned fail = 0;
  p->m = m;
  snprintf(name, sizeof name, "%s_pool%u", m->name, m->n_pools++);
  if (m->rank == 0) {
    p->data_bytes = (data_bytes + 4095) & ~(size_t)4095;
    p->map_bytes = POOL_HDR + p->data_bytes;
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)p->map_bytes) != 0 || (err = posix_fallocate(fd, 0, (off_t)p->map_bytes)) != 0) {
      logmsg(MSG_WARN, "fscl_amd: permutation pool %s (%zu MB): %s\n", name, p->map_bytes >> 20,
             strerror(err ? err : errno));
      fail = 1;
      if (fd >= 0) { close(fd); shm_unlink(name); }
    }
  }
  if (fh_shm_allgather_flags(m, &dummy, 1, 0, 0, 0, &fail) != 0)
    logmsg(MSG_FATAL, "fscl_amd: permutation pool: rank exchange failed");
  if (fail) { free(p); return NULL; }
  if (m->rank != 0) {
    struct stat sb;
    fd = shm_open(name, O_RDWR, 0600);
    if (fd < 0 || fstat(fd, &sb) != 0 || (size_t)sb.st_size <= POOL_HDR)
      logmsg(MSG_FATAL, "fscl_amd: permutation pool %s: %s", name, strerror(errno));
    p->map_bytes = (size_t)sb.st_size;
    p->data_bytes = p->map_bytes - POOL_HDR;
  }
  p->h = mmap(NULL, p->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p->h == MAP_FAILED) logmsg(MSG_FATAL, "fscl_amd: permutation pool mmap: %s", strerror(errno));
  p->data = (char *)p->h + POOL_HDR;
  if (fh_shm_barrier(m) != 0) logmsg(MSG_FATAL, "fscl_amd: permutation pool: rank exchange failed");
  if (m->rank == 0) shm_unlink(name);  /* every rank has it mapped */
  return p;
}

void fh_pool_close(fh_pool_t *p) {
  if (!p) return;
  munmap(p->h, p->map_bytes);
  free(p);
}

char *fh_pool_data(fh_pool_t *p) { return p->data; }
size_t fh_pool_bytes(const fh_pool_t *p) { return p->data_bytes; }

/* the leader: publish one trial's permutation (offsets into the data area) */
int fh_pool_publish(fh_pool_t *p, size_t rows_off, size_t nul_off, const fh_rand_t *end, unsigned long long negj) {
  const unsigned long long s = p->n_pub + 1;
  pool_pub_t *e = &p->h->ring[(s - 1) % POOL_RING];
  int r;
  if (s > POOL_RING)  /* the entry's previous publication taken by every rank */
    for (r = 1; r < p->m->world; r++)
      if (wait_ge_ull(&p->h->cons[r], s - POOL_RING) != 0) return -1;
  e->rows_off = rows_off; e->nul_off = nul_off; e->negj = negj; e->end = *end; e->seq = s;
  atomic_store_explicit(&p->h->pub, s, memory_order_release);
  p->n_pub = s;
  return 0;
}

/* the other ranks: the next publication, in order */
int fh_pool_take(fh_pool_t *p, size_t *rows_off, size_t *nul_off, fh_rand_t *end, unsigned long long *negj) {
  const unsigned long long s = p->n_take + 1;
  const pool_pub_t *e = &p->h->ring[(s - 1) % POOL_RING];
  if (wait_ge_ull(&p->h->pub, s) != 0) return -1;
  if (e->seq != s) {
    logmsg(MSG_ERROR, "fscl_amd: permutation pool: publication %llu found, %llu expected", e->seq, s);
    return -1;
  }
  *rows_off = e->rows_off; *nul_off = e->nul_off; *end = e->end; *negj = e->negj;
  atomic_store_explicit(&p->h->cons[p->m->rank], s, memory_order_release);
  p->n_take = s;
  return 0;
}

/* this rank's devices have finished reading one more row slot */
void fh_pool_release(fh_pool_t *p) {
  p->n_rel++;
  atomic_store_explicit(&p->h->rel[p->m->rank], p->n_rel, memory_order_release);
}

/* the leader: every rank has made as many releases as this one (their uploads of the
   released slots' rows are done: the buffers may be rewritten) */
int fh_pool_wait_released(fh_pool_t *p) {
  int r;
  for (r = 0; r < p->m->world; r++)
    if (r != p->m->rank && wait_ge_ull(&p->h->rel[r], p->n_rel) != 0) return -1;
  return 0;
}
