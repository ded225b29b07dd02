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
 *   AMDKUBE_DEVVIEW_ROOT   device root (default /dev)
 *   AMDKUBE_DEVVIEW_ALLOW  comma list of device paths the container was given
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

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

/* 1 when `path` names a GPU node (<root>/kfd, <root>/dri/renderD*, <root>/dri/card*) the
 * container was not given. Relative paths and other files are never hidden. */
static int hidden(const char* path) {
  if (!path || path[0] != '/') return 0;
  const char* root = getenv("AMDKUBE_DEVVIEW_ROOT");
  if (!root || !*root) root = "/dev";
  size_t rl = strlen(root);
  if (strncmp(path, root, rl) != 0 || path[rl] != '/') return 0;
  const char* rest = path + rl + 1;
  int gpu_node = strcmp(rest, "kfd") == 0 || strncmp(rest, "dri/renderD", 11) == 0 || strncmp(rest, "dri/card", 8) == 0;
  if (!gpu_node) return 0;
  return !listed(getenv("AMDKUBE_DEVVIEW_ALLOW"), path);
}

#define REAL(name, type) static type real_##name; if (!real_##name) real_##name = (type)dlsym(RTLD_NEXT, #name)

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
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real_open(path, flags, m);
}

int open64(const char* path, int flags, ...) {
  REAL(open64, open_fn);
  va_list ap;
  va_start(ap, flags);
  mode_t m = mode_arg(flags, ap);
  va_end(ap);
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real_open64(path, flags, m);
}

int openat(int dirfd, const char* path, int flags, ...) {
  REAL(openat, openat_fn);
  va_list ap;
  va_start(ap, flags);
  mode_t m = mode_arg(flags, ap);
  va_end(ap);
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real_openat(dirfd, path, flags, m);
}

int openat64(int dirfd, const char* path, int flags, ...) {
  REAL(openat64, openat_fn);
  va_list ap;
  va_start(ap, flags);
  mode_t m = mode_arg(flags, ap);
  va_end(ap);
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real_openat64(dirfd, path, flags, m);
}

/* _FORTIFY_SOURCE entry points */
int __open_2(const char* path, int flags) {
  REAL(__open_2, open2_fn);
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real___open_2(path, flags);
}

int __open64_2(const char* path, int flags) {
  REAL(__open64_2, open2_fn);
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real___open64_2(path, flags);
}

int __openat_2(int dirfd, const char* path, int flags) {
  REAL(__openat_2, openat2_fn);
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real___openat_2(dirfd, path, flags);
}

/* stat-family probes of a hidden node agree with open: it does not exist */
typedef int (*stat_fn)(const char*, struct stat*);
int stat(const char* path, struct stat* st) {
  REAL(stat, stat_fn);
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real_stat(path, st);
}

typedef int (*access_fn)(const char*, int);
int access(const char* path, int mode) {
  REAL(access, access_fn);
  if (hidden(path)) { errno = ENOENT; return -1; }
  return real_access(path, mode);
}
