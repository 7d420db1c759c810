/*
 * sr_spec.c -- code objects of the shape-specialised sweep kernel (host side, no GPU).
 *
 * A session with LDS columns runs its sweep kernel compiled for the dataset's exact shape (sites,
 * taxa, hard sites fixed at compile time: layout offsets, strides, loop bounds and uniform_int
 * divisors become immediates).  This file finds that code object in the cache or
 * compiles it:
 *   - sources: build/spec/, the snapshot of csrc/ that `make` copies next to libseriation.so
 *     together with the library itself, so a kernel is always compiled from exactly the sources
 *     the loaded library was built from; their FNV-1a hash is compiled into the library
 *     (SR_SPEC_HASH, computed by this file's tool build) and re-checked before any compile;
 *   - cache: $SR_JIT_CACHE, else build/jit/ beside the snapshot; the file name is the hash of
 *     the snapshot, the definitions, the flags, the target, and the compiler's ROCm version;
 *   - compile: `hipcc --genco` in a child process (posix_spawn, output to a log), never while a
 *     profiler tool library is preloaded (its library would initialise the GPU in every process
 *     of the compiler's exec chain): then the cache alone serves, else the generic kernel runs.
 *   - embedded: the shapes of csrc/sr_embed_shapes.txt (the reference's datasets, the bench matrix)
 *     are compiled by `make` (build/srembed, this machinery with the cache in build/emb/) and linked
 *     into libseriation.so itself (build/sr_emb.c); a session of such a shape loads its code object
 *     from the library's memory -- no compiler, no cache, no snapshot needed at run time.
 * sr_specialize() (sr_device.hip) fills the cache ahead of time without a GPU for other shapes;
 * __graft_entry__.build() does so for the GPU tests' shapes.
 *
 * Built with -DSR_SPEC_TOOL it is the build's hash tool: `srhash <dir>` prints the snapshot hash.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <spawn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include "sr_internal.h"

extern char **environ;

/* the snapshot, in hashing order (names only: build/spec/ is flat) */
static const char *const spec_files[] = {"sr_device.hip", "sr_math.h", "sr_rng.h", "sr_tables.h", "sr_internal.h",
                                         "seriation.h"};
#define SPEC_NFILES (sizeof spec_files / sizeof spec_files[0])
#define SPEC_FLAGS "--genco -O3 -std=c++17 -ffp-contract=off -fno-fast-math -mllvm -disable-machine-licm"   /* as the Makefile's HIPFLAGS */

static uint64_t fnv(uint64_t h, const void *p, size_t n)
{
  const unsigned char *b = (const unsigned char *)p;
  for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
  return h;
}

static int hash_file(const char *path, uint64_t *h)
{
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  unsigned char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) *h = fnv(*h, buf, n);
  const int bad = ferror(f);
  fclose(f);
  return bad ? -1 : 0;
}

/* FNV-1a over (name, contents) of every snapshot file */
static int hash_snapshot(const char *dir, uint64_t *out)
{
  uint64_t h = 1469598103934665603ull;
  char p[4400];
  for (size_t i = 0; i < SPEC_NFILES; ++i) {
    h = fnv(h, spec_files[i], strlen(spec_files[i]) + 1);
    snprintf(p, sizeof p, "%s/%s", dir, spec_files[i]);
    if (hash_file(p, &h) != 0) return -1;
  }
  *out = h;
  return 0;
}

#ifdef SR_SPEC_TOOL
int main(int argc, char **argv)
{
  uint64_t h;
  if (argc != 2 || hash_snapshot(argv[1], &h) != 0) {
    fprintf(stderr, "usage: srhash <snapshot dir> (all of sr_device.hip sr_math.h sr_rng.h sr_tables.h "
                    "sr_internal.h seriation.h readable)\n");
    return 1;
  }
  printf("%016llx\n", (unsigned long long)h);
  return 0;
}
#else

#ifndef SR_ARCH
#define SR_ARCH "gfx950"
#endif
/* extra device definitions of an experimental library build (tools/build_variant.sh): its specialised
   kernels are compiled with them too (they are part of the key) */
#ifndef SR_SPEC_EXTRA
#define SR_SPEC_EXTRA ""
#endif

/* resolved once per process: the library's directory, its snapshot and whether it is intact */
static struct {
  char libdir[4096];
  char snap[4200];
  uint64_t src_hash;
  char rocm[128];
  int state;   /* 0 ok; SR_SPEC_ENOSRC / SR_SPEC_ESTALE */
} g_spec;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static pthread_mutex_t g_msg_lock = PTHREAD_MUTEX_INITIALIZER;
static unsigned g_msg_seen;   /* reasons already reported (one stderr line per reason and process) */

static const char *hipcc_path(void)
{
  const char *e = getenv("SR_HIPCC");
  return (e && *e) ? e : "/opt/rocm/bin/hipcc";
}

/* the compiler's ROCm version: <hipcc>/../.info/version (a ROCm upgrade changes every key) */
static void rocm_version(char *out, size_t len)
{
  char p[4200];
  snprintf(p, sizeof p, "%s", hipcc_path());
  char *sl = strrchr(p, '/');
  out[0] = 0;
  if (sl) {
    *sl = 0;
    char v[4300];
    snprintf(v, sizeof v, "%s/../.info/version", p);
    FILE *f = fopen(v, "r");
    if (f) {
      if (fgets(out, (int)len, f)) out[strcspn(out, "\r\n")] = 0;
      fclose(f);
    }
  }
  if (!out[0]) {   /* no version file: the compiler binary's identity */
    struct stat st;
    if (stat(hipcc_path(), &st) == 0)
      snprintf(out, len, "hipcc:%lld:%lld", (long long)st.st_size, (long long)st.st_mtime);
    else
      snprintf(out, len, "hipcc:absent");
  }
}

static void spec_init(void)
{
  Dl_info info;
  g_spec.state = SR_SPEC_ENOSRC;
  if (!dladdr((void *)&spec_init, &info) || !info.dli_fname) return;
  snprintf(g_spec.libdir, sizeof g_spec.libdir, "%s", info.dli_fname);
  rocm_version(g_spec.rocm, sizeof g_spec.rocm);
  /* spec/ next to the library, else next to its directory (the test builds in build/force/ etc. share
     build/spec/); the cache directory sits beside the snapshot */
  for (int up = 0; up < 2; ++up) {
    char *sl = strrchr(g_spec.libdir, '/');
    if (!sl) return;
    *sl = 0;
    snprintf(g_spec.snap, sizeof g_spec.snap, "%s/spec", g_spec.libdir);
    if (hash_snapshot(g_spec.snap, &g_spec.src_hash) == 0) break;
    if (up == 1) return;
  }
#ifdef SR_SPEC_HASH
  if (g_spec.src_hash != (uint64_t)SR_SPEC_HASH) { g_spec.state = SR_SPEC_ESTALE; return; }
#endif
  g_spec.state = 0;
}

const char *sr_spec_reason(int code)
{
  switch (code) {
    case SR_SPEC_ENOSRC: return "no kernel source snapshot next to the library (build/spec/)";
    case SR_SPEC_ESTALE: return "the source snapshot differs from the sources the library was built from (rebuild)";
    case SR_SPEC_ENOCC: return "no compiler (SR_HIPCC / /opt/rocm/bin/hipcc) and no cached code object";
    case SR_SPEC_ECC: return "the compile failed";
    case SR_SPEC_EPROF: return "a profiler tool library is preloaded and the code object is not cached";
    case SR_SPEC_ELOAD: return "the code object did not load or does not match this library";
    case SR_SPEC_ECACHE: return "the cache directory cannot be created or written ($SR_JIT_CACHE / build/jit)";
    case SR_SPEC_ENOJIT: return "not embedded, not in the cache, and SR_JIT=cache forbids compiling at run time "
                                "(sr_specialize fills the cache ahead)";
    default: return "unknown";
  }
}

void sr_spec_note(int code, const char *detail)
{
  char log[4608];
  const size_t n = detail ? strlen(detail) : 0;
  if (code == SR_SPEC_ECC && n > 3 && !strcmp(detail + n - 3, ".co") && n < sizeof log - 2) {
    snprintf(log, sizeof log, "see %.*s.log", (int)(n - 3), detail);   /* the compiler's output */
    detail = log;
  }
  const unsigned bit = 1u << ((unsigned)(-code) & 15u);
  pthread_mutex_lock(&g_msg_lock);
  const int first = !(g_msg_seen & bit);
  g_msg_seen |= bit;
  pthread_mutex_unlock(&g_msg_lock);
  if (first)
    fprintf(stderr, "seriation: shape-specialised kernel unavailable: %s%s%s; the generic kernel runs\n",
            sr_spec_reason(code), detail ? ": " : "", detail ? detail : "");
}

/* a profiler's tool library in this process (rocprofv3 / rocprofiler-sdk set these) */
static int profiler_preloaded(void)
{
  const char *p = getenv("LD_PRELOAD");
  if (p && strstr(p, "rocprof")) return 1;
  for (char **e = environ; e && *e; ++e)
    if (!strncmp(*e, "ROCP_TOOL_LIBRARIES=", 20) || !strncmp(*e, "ROCPROF", 7) || !strncmp(*e, "HSA_TOOLS_LIB=", 14))
      return 1;
  return 0;
}

static void defs_of(const sr_spec_shape *s, char *defs, size_t len)
{
  snprintf(defs, len, "-DSR_JIT -DSR_JIT_TB=%d -DSR_JIT_NWM=%d -DSR_FN=%d -DSR_FM=%d -DSR_FH=%d%s%s%s", s->TB, s->NWM,
           s->N, s->M, s->NH, s->force ? " -DSR_FORCE_EXACT" : "", SR_SPEC_EXTRA[0] ? " " : "", SR_SPEC_EXTRA);
}

static void cache_dir(char *dir, size_t len)
{
  const char *e = getenv("SR_JIT_CACHE");
  if (e && *e) snprintf(dir, len, "%s", e);
  else snprintf(dir, len, "%s/jit", g_spec.libdir);
}

int sr_spec_path(const sr_spec_shape *s, char *path, size_t len)
{
  pthread_once(&g_once, spec_init);
  if (g_spec.state) return g_spec.state;
  char defs[1024], dir[4200];
  defs_of(s, defs, sizeof defs);
  uint64_t h = g_spec.src_hash;
  h = fnv(h, defs, strlen(defs) + 1);
  h = fnv(h, SPEC_FLAGS, sizeof SPEC_FLAGS);
  h = fnv(h, SR_ARCH, sizeof SR_ARCH);
  h = fnv(h, g_spec.rocm, strlen(g_spec.rocm) + 1);
  cache_dir(dir, sizeof dir);
  if ((size_t)snprintf(path, len, "%s/sr_%016llx.co", dir, (unsigned long long)h) >= len) return SR_SPEC_ENOSRC;
  return 0;
}

static void mkdirs(const char *dir)
{
  char p[4200];
  snprintf(p, sizeof p, "%s", dir);
  for (char *q = p + 1; *q; ++q)
    if (*q == '/') { *q = 0; (void)mkdir(p, 0755); *q = '/'; }
  (void)mkdir(p, 0755);
}

extern const sr_spec_emb sr_spec_emb_table[] __attribute__((weak, visibility("hidden")));
extern const int sr_spec_emb_count __attribute__((weak, visibility("hidden")));

const void *sr_spec_embedded(const sr_spec_shape *s, size_t *bytes)
{
  if (!&sr_spec_emb_count || !sr_spec_emb_table) return NULL;
  for (int k = 0; k < sr_spec_emb_count; ++k) {
    const sr_spec_emb *e = &sr_spec_emb_table[k];
    if (e->TB == s->TB && e->NWM == s->NWM && e->N == s->N && e->M == s->M && e->NH == s->NH && e->force == s->force) {
      *bytes = (size_t)(e->end - e->begin);
      return e->begin;
    }
  }
  return NULL;
}

int sr_spec_object(const sr_spec_shape *s, char *path, size_t len, int announce)
{
  int rc = sr_spec_path(s, path, len);
  if (rc) return rc;
  if (access(path, R_OK) == 0) return 0;
  if (profiler_preloaded()) return SR_SPEC_EPROF;
  const char *cc = hipcc_path();
  if (access(cc, X_OK) != 0) return SR_SPEC_ENOCC;
  char dir[4200], tmp[4500], log[4500], inc[4300], src[4300], arch[64], defs[1024], fl[1280];
  snprintf(dir, sizeof dir, "%s", path);
  char *sl = strrchr(dir, '/');
  if (sl) *sl = 0;
  mkdirs(dir);
  if (access(dir, W_OK) != 0) return SR_SPEC_ECACHE;
  /* a per-compile temporary name: shard threads and processes may compile the same shape together;
     rename() publishes the finished object atomically */
  static int seq;
  snprintf(tmp, sizeof tmp, "%s.%d.%d.tmp", path, (int)getpid(), __atomic_add_fetch(&seq, 1, __ATOMIC_RELAXED));
  snprintf(log, sizeof log, "%.*s.log", (int)(strlen(path) - 3), path);
  snprintf(inc, sizeof inc, "-I%s", g_spec.snap);
  snprintf(src, sizeof src, "%s/sr_device.hip", g_spec.snap);
  snprintf(arch, sizeof arch, "--offload-arch=%s", SR_ARCH);
  defs_of(s, defs, sizeof defs);
  snprintf(fl, sizeof fl, "%s %s", SPEC_FLAGS, defs);
  if (announce)
    fprintf(stderr, "seriation: compiling the sweep kernel specialised for %d sites x %d taxa, %d hard sites (once: "
                    "cached in %s)\n", s->N, s->M, s->NH, dir);
  char *argv[48];
  int na = 0;
  argv[na++] = (char *)cc;
  argv[na++] = arch;
  char *sv = NULL;
  for (char *t = strtok_r(fl, " ", &sv); t && na < 40; t = strtok_r(NULL, " ", &sv)) argv[na++] = t;
  argv[na++] = inc;
  argv[na++] = (char *)"-o";
  argv[na++] = tmp;
  argv[na++] = src;
  argv[na] = NULL;
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  posix_spawn_file_actions_addopen(&fa, 1, log, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  posix_spawn_file_actions_adddup2(&fa, 1, 2);
  pid_t pid;
  const int sr = posix_spawn(&pid, cc, &fa, NULL, argv, environ);
  posix_spawn_file_actions_destroy(&fa);
  if (sr != 0) return SR_SPEC_ENOCC;
  int st = 0;
  while (waitpid(pid, &st, 0) < 0)
    if (errno != EINTR) return SR_SPEC_ECC;
  if (!WIFEXITED(st) || WEXITSTATUS(st) != 0 || rename(tmp, path) != 0) {
    (void)unlink(tmp);
    return SR_SPEC_ECC;
  }
  return 0;
}
#endif
