/* libamdkube-devview.so — the container's view of GPU device nodes under a Landlock guard.
 *
 * Under `isolation=landlock` (an unprivileged node: no mount namespace to hide nodes in) the
 * kernel refuses every /dev/dri node and /dev/kfd the container was not given, with EACCES
 * (devguard.h). ROCr's thunk reads a refused render node as a fatal error
 * (hsa_init → HSA_STATUS_ERROR_OUT_OF_RESOURCES, measured on MI355X:
 * profiles/r3/isolation.md), while a node that is absent (ENOENT) — what Docker's --device and
 * the reference's HostConfig.Devices produce (pkg/kubelet/dockershim/docker_container.go:155-172)
 * — is skipped. This preload turns "not in the container's device list" into ENOENT before the
 * kernel is asked, so a GPU container sees exactly its own GPUs, as it would with a private
 * /dev/dri. It enforces nothing: a process that bypasses it (static binary, raw syscall,
 * LD_PRELOAD cleared) still meets the kernel's EACCES.
 *
 * Covered: every open entry point (open/openat/…64, the _FORTIFY_SOURCE __open*_2 ones, fopen,
 * fopen64), every stat-family probe (stat/lstat/…64, fstatat/…64, statx and the pre-2.33 glibc
 * __xstat/__lxstat/__fxstatat exports), access/faccessat/euidaccess, and directory enumeration
 * of <root>/dri (readdir/readdir64 of a DIR* opened on it, scandir/scandir64, glob/glob64 — a
 * libdrm-style walk of /dev/dri lists only the container's nodes). Paths relative to a dirfd
 * or the cwd are resolved before the check.
 *
 *   AMDKUBE_DEVVIEW_ROOT   device root (default /dev)
 *   AMDKUBE_DEVVIEW_ALLOW  comma list of device paths the container was given
 */
#define _GNU_SOURCE
#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <glob.h>
#include <limits.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

/* bind dlsym/dlvsym to their original version, not glibc 2.34's: the preload must also load into
 * images whose glibc predates 2.34 */
__asm__(".symver dlsym,dlsym@GLIBC_2.2.5");
__asm__(".symver dlvsym,dlvsym@GLIBC_2.2.5");

static int listed(const char* list, const char* path) {
  size_t n = strlen(path);
  const char* p = list;
  while (p && *p) {
    const char* e = strchr(p, ',');
    size_t len = e ? (size_t)(e - p) : strlen(p);
    if (len == n && strncmp(p, path, n) == 0) return 1;
    p = e ? e + 1 : NULL;
  }
  return 0;
}

/* the launcher (amdkube-nsexec) must see every node to build its Landlock ruleset: the view is
 * off in it even when it was started with the preload */
static int g_off;
__attribute__((constructor)) static void devview_init(void) {
  g_off = strcmp(program_invocation_short_name, "amdkube-nsexec") == 0;
}

static const char* dev_root(size_t* rl) {
  const char* root = getenv("AMDKUBE_DEVVIEW_ROOT");
  if (!root || !*root) root = "/dev";
  *rl = strlen(root);
  while (*rl > 1 && root[*rl - 1] == '/') (*rl)--;
  return root;
}

/* 1 when the absolute `path` names a GPU node (<root>/kfd, <root>/dri/renderD*,
 * <root>/dri/card*) the container was not given. Other files are never hidden. */
static int hidden_abs(const char* path) {
  if (g_off || !path || path[0] != '/') return 0;
  size_t rl;
  const char* root = dev_root(&rl);
  if (strncmp(path, root, rl) != 0 || path[rl] != '/') return 0;
  const char* rest = path + rl + 1;
  while (*rest == '/') rest++;
  int gpu_node = strcmp(rest, "kfd") == 0 || strncmp(rest, "dri/renderD", 11) == 0 || strncmp(rest, "dri/card", 8) == 0;
  if (!gpu_node) {
    /* <root>/dri/by-path/… links name the same nodes: judge them by what they resolve to */
    if (strncmp(rest, "dri/", 4) != 0) return 0;
    char real[PATH_MAX];
    if (!realpath(path, real) || strcmp(real, path) == 0) return 0;
    return hidden_abs(real);
  }
  char canon[PATH_MAX];
  snprintf(canon, sizeof canon, "%.*s/%s", (int)rl, root, rest);
  return !listed(getenv("AMDKUBE_DEVVIEW_ALLOW"), canon);
}

/* The absolute form of `path` taken relative to `dirfd` (AT_FDCWD: the cwd). */
static const char* at_path(int dirfd, const char* path, char* buf, size_t n) {
  if (!path || !*path || path[0] == '/') return path;
  char dir[PATH_MAX];
  if (dirfd == AT_FDCWD) {
    if (!getcwd(dir, sizeof dir)) return path;
  } else {
    char link[64];
    snprintf(link, sizeof link, "/proc/self/fd/%d", dirfd);
    ssize_t k = readlink(link, dir, sizeof dir - 1);
    if (k <= 0) return path;
    dir[k] = 0;
  }
  const char* p = path;
  while (p[0] == '.' && p[1] == '/') p += 2;
  int w = snprintf(buf, n, "%s/%s", strcmp(dir, "/") == 0 ? "" : dir, p);
  return (w < 0 || (size_t)w >= n) ? path : buf;
}

static int hidden_at(int dirfd, const char* path) {
  if (!path) return 0;
  char buf[PATH_MAX];
  return hidden_abs(at_path(dirfd, path, buf, sizeof buf));
}

static int hidden(const char* path) { return hidden_at(AT_FDCWD, path); }

#define REAL(name, type) static type real_##name; if (!real_##name) real_##name = (type)dlsym(RTLD_NEXT, #name)
/* the pre-2.33 stat exports exist only as compat symbols on a newer glibc: dlsym does not see
 * them, dlvsym at the x86-64 base version does */
#define REAL_COMPAT(name, type)                                                         \
  static type real_##name;                                                              \
  if (!real_##name) real_##name = (type)dlsym(RTLD_NEXT, #name);                        \
  if (!real_##name) real_##name = (type)dlvsym(RTLD_NEXT, #name, "GLIBC_2.2.5");        \
  if (!real_##name) { errno = ENOSYS; return -1; }
#define ABSENT(cond) do { if (cond) { errno = ENOENT; return -1; } } while (0)

typedef int (*open_fn)(const char*, int, ...);
typedef int (*openat_fn)(int, const char*, int, ...);
typedef int (*open2_fn)(const char*, int);
typedef int (*openat2_fn)(int, const char*, int);

static mode_t mode_arg(int flags, va_list ap) {
  return (flags & O_CREAT) || (flags & O_TMPFILE) == O_TMPFILE ? (mode_t)va_arg(ap, int) : 0;
}

int open(const char* path, int flags, ...) {
  REAL(open, open_fn);
  va_list ap;
  va_start(ap, flags);
  mode_t m = mode_arg(flags, ap);
  va_end(ap);
  ABSENT(hidden(path));
  return real_open(path, flags, m);
}

int open64(const char* path, int flags, ...) {
  REAL(open64, open_fn);
  va_list ap;
  va_start(ap, flags);
  mode_t m = mode_arg(flags, ap);
  va_end(ap);
  ABSENT(hidden(path));
  return real_open64(path, flags, m);
}

int openat(int dirfd, const char* path, int flags, ...) {
  REAL(openat, openat_fn);
  va_list ap;
  va_start(ap, flags);
  mode_t m = mode_arg(flags, ap);
  va_end(ap);
  ABSENT(hidden_at(dirfd, path));
  return real_openat(dirfd, path, flags, m);
}

int openat64(int dirfd, const char* path, int flags, ...) {
  REAL(openat64, openat_fn);
  va_list ap;
  va_start(ap, flags);
  mode_t m = mode_arg(flags, ap);
  va_end(ap);
  ABSENT(hidden_at(dirfd, path));
  return real_openat64(dirfd, path, flags, m);
}

/* _FORTIFY_SOURCE entry points */
int __open_2(const char* path, int flags) {
  REAL(__open_2, open2_fn);
  ABSENT(hidden(path));
  return real___open_2(path, flags);
}

int __open64_2(const char* path, int flags) {
  REAL(__open64_2, open2_fn);
  ABSENT(hidden(path));
  return real___open64_2(path, flags);
}

int __openat_2(int dirfd, const char* path, int flags) {
  REAL(__openat_2, openat2_fn);
  ABSENT(hidden_at(dirfd, path));
  return real___openat_2(dirfd, path, flags);
}

int __openat64_2(int dirfd, const char* path, int flags) {
  REAL(__openat64_2, openat2_fn);
  ABSENT(hidden_at(dirfd, path));
  return real___openat64_2(dirfd, path, flags);
}

/* stdio opens go through glibc-internal open calls the preload cannot see */
typedef FILE* (*fopen_fn)(const char*, const char*);
FILE* fopen(const char* path, const char* mode) {
  REAL(fopen, fopen_fn);
  if (hidden(path)) { errno = ENOENT; return NULL; }
  return real_fopen(path, mode);
}

FILE* fopen64(const char* path, const char* mode) {
  REAL(fopen64, fopen_fn);
  if (hidden(path)) { errno = ENOENT; return NULL; }
  return real_fopen64(path, mode);
}

/* stat-family probes of a hidden node agree with open: it does not exist */
typedef int (*stat_fn)(const char*, struct stat*);
typedef int (*stat64_fn)(const char*, struct stat64*);
typedef int (*fstatat_fn)(int, const char*, struct stat*, int);
typedef int (*fstatat64_fn)(int, const char*, struct stat64*, int);
typedef int (*statx_fn)(int, const char*, int, unsigned int, struct statx*);
typedef int (*xstat_fn)(int, const char*, struct stat*);
typedef int (*xstat64_fn)(int, const char*, struct stat64*);
typedef int (*fxstatat_fn)(int, int, const char*, struct stat*, int);
typedef int (*fxstatat64_fn)(int, int, const char*, struct stat64*, int);

int stat(const char* path, struct stat* st) {
  REAL(stat, stat_fn);
  ABSENT(hidden(path));
  return real_stat(path, st);
}

int stat64(const char* path, struct stat64* st) {
  REAL(stat64, stat64_fn);
  ABSENT(hidden(path));
  return real_stat64(path, st);
}

int lstat(const char* path, struct stat* st) {
  REAL(lstat, stat_fn);
  ABSENT(hidden(path));
  return real_lstat(path, st);
}

int lstat64(const char* path, struct stat64* st) {
  REAL(lstat64, stat64_fn);
  ABSENT(hidden(path));
  return real_lstat64(path, st);
}

int fstatat(int dirfd, const char* path, struct stat* st, int flags) {
  REAL(fstatat, fstatat_fn);
  ABSENT(hidden_at(dirfd, path));
  return real_fstatat(dirfd, path, st, flags);
}

int fstatat64(int dirfd, const char* path, struct stat64* st, int flags) {
  REAL(fstatat64, fstatat64_fn);
  ABSENT(hidden_at(dirfd, path));
  return real_fstatat64(dirfd, path, st, flags);
}

int statx(int dirfd, const char* path, int flags, unsigned int mask, struct statx* st) {
  REAL(statx, statx_fn);
  ABSENT(hidden_at(dirfd, path));
  return real_statx(dirfd, path, flags, mask, st);
}

/* glibc before 2.33 exports these and its stat() macros call them */
int __xstat(int ver, const char* path, struct stat* st) {
  REAL_COMPAT(__xstat, xstat_fn)
  ABSENT(hidden(path));
  return real___xstat(ver, path, st);
}

int __xstat64(int ver, const char* path, struct stat64* st) {
  REAL_COMPAT(__xstat64, xstat64_fn)
  ABSENT(hidden(path));
  return real___xstat64(ver, path, st);
}

int __lxstat(int ver, const char* path, struct stat* st) {
  REAL_COMPAT(__lxstat, xstat_fn)
  ABSENT(hidden(path));
  return real___lxstat(ver, path, st);
}

int __lxstat64(int ver, const char* path, struct stat64* st) {
  REAL_COMPAT(__lxstat64, xstat64_fn)
  ABSENT(hidden(path));
  return real___lxstat64(ver, path, st);
}

int __fxstatat(int ver, int dirfd, const char* path, struct stat* st, int flags) {
  REAL_COMPAT(__fxstatat, fxstatat_fn)
  ABSENT(hidden_at(dirfd, path));
  return real___fxstatat(ver, dirfd, path, st, flags);
}

int __fxstatat64(int ver, int dirfd, const char* path, struct stat64* st, int flags) {
  REAL_COMPAT(__fxstatat64, fxstatat64_fn)
  ABSENT(hidden_at(dirfd, path));
  return real___fxstatat64(ver, dirfd, path, st, flags);
}

typedef int (*access_fn)(const char*, int);
typedef int (*faccessat_fn)(int, const char*, int, int);
int access(const char* path, int mode) {
  REAL(access, access_fn);
  ABSENT(hidden(path));
  return real_access(path, mode);
}

int faccessat(int dirfd, const char* path, int mode, int flags) {
  REAL(faccessat, faccessat_fn);
  ABSENT(hidden_at(dirfd, path));
  return real_faccessat(dirfd, path, mode, flags);
}

int euidaccess(const char* path, int mode) {
  REAL(euidaccess, access_fn);
  ABSENT(hidden(path));
  return real_euidaccess(path, mode);
}

int eaccess(const char* path, int mode) {
  REAL(eaccess, access_fn);
  ABSENT(hidden(path));
  return real_eaccess(path, mode);
}

/* ---------------------------------------------------------------- enumeration of <root>/dri
 * A DIR* opened on the dri directory is remembered (a small table, lock-protected); readdir on
 * it skips the nodes hidden_abs() hides, so a walk lists only the container's devices. */
#define MAX_DIRS 64
static struct { DIR* d; char path[PATH_MAX]; } g_dirs[MAX_DIRS];
static pthread_mutex_t g_dirs_mu = PTHREAD_MUTEX_INITIALIZER;

static int is_dri_dir(const char* abs) {
  if (g_off) return 0;
  size_t rl;
  const char* root = dev_root(&rl);
  if (!abs || strncmp(abs, root, rl) != 0 || abs[rl] != '/') return 0;
  const char* rest = abs + rl + 1;
  return strcmp(rest, "dri") == 0 || strcmp(rest, "dri/") == 0;
}

static void remember(DIR* d, const char* abs) {
  pthread_mutex_lock(&g_dirs_mu);
  for (int i = 0; i < MAX_DIRS; i++)
    if (!g_dirs[i].d) {
      g_dirs[i].d = d;
      snprintf(g_dirs[i].path, sizeof g_dirs[i].path, "%s", abs);
      break;
    }
  pthread_mutex_unlock(&g_dirs_mu);
}

/* copies the remembered directory of `d` into `out`; 0 when `d` is not a dri walk */
static int dri_dir_of(DIR* d, char* out, size_t n) {
  int found = 0;
  pthread_mutex_lock(&g_dirs_mu);
  for (int i = 0; i < MAX_DIRS; i++)
    if (g_dirs[i].d == d) {
      snprintf(out, n, "%s", g_dirs[i].path);
      found = 1;
      break;
    }
  pthread_mutex_unlock(&g_dirs_mu);
  return found;
}

static int entry_hidden(const char* dir, const char* name) {
  char full[PATH_MAX];
  size_t dl = strlen(dir);
  snprintf(full, sizeof full, "%.*s/%s", (int)(dl && dir[dl - 1] == '/' ? dl - 1 : dl), dir, name);
  return hidden_abs(full);
}

typedef DIR* (*opendir_fn)(const char*);
typedef DIR* (*fdopendir_fn)(int);
typedef int (*closedir_fn)(DIR*);
typedef struct dirent* (*readdir_fn)(DIR*);
typedef struct dirent64* (*readdir64_fn)(DIR*);

DIR* opendir(const char* path) {
  REAL(opendir, opendir_fn);
  DIR* d = real_opendir(path);
  char buf[PATH_MAX];
  const char* abs = at_path(AT_FDCWD, path, buf, sizeof buf);
  if (d && is_dri_dir(abs)) remember(d, abs);
  return d;
}

DIR* fdopendir(int fd) {
  REAL(fdopendir, fdopendir_fn);
  DIR* d = real_fdopendir(fd);
  char buf[PATH_MAX];
  const char* abs = at_path(fd, ".", buf, sizeof buf);
  if (d && abs) {
    size_t n = strlen(abs);
    if (n >= 2 && strcmp(abs + n - 2, "/.") == 0) buf[n - 2] = 0;
    if (is_dri_dir(buf)) remember(d, buf);
  }
  return d;
}

int closedir(DIR* d) {
  REAL(closedir, closedir_fn);
  pthread_mutex_lock(&g_dirs_mu);
  for (int i = 0; i < MAX_DIRS; i++)
    if (g_dirs[i].d == d) g_dirs[i].d = NULL;
  pthread_mutex_unlock(&g_dirs_mu);
  return real_closedir(d);
}

struct dirent* readdir(DIR* d) {
  REAL(readdir, readdir_fn);
  char dir[PATH_MAX];
  int dri = dri_dir_of(d, dir, sizeof dir);
  struct dirent* e;
  while ((e = real_readdir(d)) && dri && entry_hidden(dir, e->d_name)) {
  }
  return e;
}

struct dirent64* readdir64(DIR* d) {
  REAL(readdir64, readdir64_fn);
  char dir[PATH_MAX];
  int dri = dri_dir_of(d, dir, sizeof dir);
  struct dirent64* e;
  while ((e = real_readdir64(d)) && dri && entry_hidden(dir, e->d_name)) {
  }
  return e;
}

/* scandir and glob walk directories through glibc-internal calls: filter their results */
typedef int (*scandir_fn)(const char*, struct dirent***, int (*)(const struct dirent*),
                          int (*)(const struct dirent**, const struct dirent**));
typedef int (*scandir64_fn)(const char*, struct dirent64***, int (*)(const struct dirent64*),
                            int (*)(const struct dirent64**, const struct dirent64**));

int scandir(const char* path, struct dirent*** list, int (*sel)(const struct dirent*),
            int (*cmp)(const struct dirent**, const struct dirent**)) {
  REAL(scandir, scandir_fn);
  int n = real_scandir(path, list, sel, cmp);
  char buf[PATH_MAX];
  const char* abs = at_path(AT_FDCWD, path, buf, sizeof buf);
  if (n <= 0 || !is_dri_dir(abs)) return n;
  int k = 0;
  for (int i = 0; i < n; i++) {
    if (entry_hidden(abs, (*list)[i]->d_name)) free((*list)[i]);
    else (*list)[k++] = (*list)[i];
  }
  return k;
}

int scandir64(const char* path, struct dirent64*** list, int (*sel)(const struct dirent64*),
              int (*cmp)(const struct dirent64**, const struct dirent64**)) {
  REAL(scandir64, scandir64_fn);
  int n = real_scandir64(path, list, sel, cmp);
  char buf[PATH_MAX];
  const char* abs = at_path(AT_FDCWD, path, buf, sizeof buf);
  if (n <= 0 || !is_dri_dir(abs)) return n;
  int k = 0;
  for (int i = 0; i < n; i++) {
    if (entry_hidden(abs, (*list)[i]->d_name)) free((*list)[i]);
    else (*list)[k++] = (*list)[i];
  }
  return k;
}

typedef int (*glob_fn)(const char*, int, int (*)(const char*, int), glob_t*);
typedef int (*glob64_fn)(const char*, int, int (*)(const char*, int), glob64_t*);

/* drop hidden paths from a glob result (glob_t and glob64_t share their layout of names) */
#define FILTER_GLOB(rc, g)                                                     \
  do {                                                                         \
    if ((rc) != 0 || !(g) || !(g)->gl_pathv) return (rc);                      \
    size_t start = (g)->gl_offs, k = start;                                    \
    for (size_t i = start; i < start + (g)->gl_pathc; i++) {                   \
      char* p = (g)->gl_pathv[i];                                              \
      char buf[PATH_MAX];                                                      \
      if (hidden_abs(at_path(AT_FDCWD, p, buf, sizeof buf))) free(p);          \
      else (g)->gl_pathv[k++] = p;                                             \
    }                                                                          \
    (g)->gl_pathc = k - start;                                                 \
    (g)->gl_pathv[k] = NULL;                                                   \
    return (g)->gl_pathc ? 0 : GLOB_NOMATCH;                                   \
  } while (0)

int glob(const char* pat, int flags, int (*errfn)(const char*, int), glob_t* g) {
  REAL(glob, glob_fn);
  int rc = real_glob(pat, flags, errfn, g);
  FILTER_GLOB(rc, g);
}

int glob64(const char* pat, int flags, int (*errfn)(const char*, int), glob64_t* g) {
  REAL(glob64, glob64_fn);
  int rc = real_glob64(pat, flags, errfn, g);
  FILTER_GLOB(rc, g);
}
