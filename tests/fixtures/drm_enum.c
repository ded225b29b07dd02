/* A libdrm/ROCr-style enumeration of a device root, used by tests/test_isolation.py: walk
 * <root>/dri with readdir, scandir and glob(3), then probe every render node the walks could
 * have seen (and every renderD128..135 by name) with stat64/lstat/statx/faccessat/fopen/
 * open/openat-relative. Prints one JSON object: {"readdir": [...], "scandir": [...],
 * "glob": [...], "probe": {"renderD128": {"stat64": "ok"|strerror, ...}, ...}}. */
#define _GNU_SOURCE
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <glob.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

static const char* res(int rc) { return rc == 0 ? "ok" : strerror(errno); }

static int cmpstr(const void* a, const void* b) { return strcmp(*(char* const*)a, *(char* const*)b); }

static void print_list(const char* key, char** v, int n) {
  qsort(v, n, sizeof(char*), cmpstr);
  printf("\"%s\": [", key);
  for (int i = 0; i < n; i++) printf("%s\"%s\"", i ? ", " : "", v[i]);
  printf("]");
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* root = argv[1];
  char dri[4096], path[4096];
  snprintf(dri, sizeof dri, "%s/dri", root);
  char* names[256];
  int n = 0;
  printf("{");
  DIR* d = opendir(dri);
  struct dirent* e;
  while (d && (e = readdir(d)) && n < 256)
    if (e->d_name[0] != '.') names[n++] = strdup(e->d_name);
  if (d) closedir(d);
  print_list("readdir", names, n);
  struct dirent** list = NULL;
  int m = scandir(dri, &list, NULL, alphasort);
  n = 0;
  for (int i = 0; i < m; i++)
    if (list[i]->d_name[0] != '.') names[n++] = list[i]->d_name;
  printf(", ");
  print_list("scandir", names, n);
  glob_t g;
  snprintf(path, sizeof path, "%s/renderD*", dri);
  int grc = glob(path, 0, NULL, &g);
  n = 0;
  for (size_t i = 0; grc == 0 && i < g.gl_pathc; i++) names[n++] = strrchr(g.gl_pathv[i], '/') + 1;
  printf(", ");
  print_list("glob", names, n);
  printf(", \"probe\": {");
  int dirfd = open(dri, O_RDONLY | O_DIRECTORY);
  for (int minor = 128; minor < 136; minor++) {
    snprintf(path, sizeof path, "%s/renderD%d", dri, minor);
    char rel[64];
    snprintf(rel, sizeof rel, "renderD%d", minor);
    struct stat64 s64;
    struct stat st;
    struct statx sx;
    printf("%s\"renderD%d\": {", minor > 128 ? ", " : "", minor);
    printf("\"stat64\": \"%s\"", res(stat64(path, &s64)));
    printf(", \"lstat\": \"%s\"", res(lstat(path, &st)));
    printf(", \"statx\": \"%s\"", res(statx(AT_FDCWD, path, 0, STATX_BASIC_STATS, &sx)));
    printf(", \"fstatat_rel\": \"%s\"", res(fstatat(dirfd, rel, &st, 0)));
    printf(", \"faccessat\": \"%s\"", res(faccessat(AT_FDCWD, path, R_OK | W_OK, 0)));
    FILE* f = fopen(path, "r+");
    printf(", \"fopen\": \"%s\"", f ? "ok" : strerror(errno));
    if (f) fclose(f);
    int fd = open(path, O_RDWR);
    printf(", \"open\": \"%s\"", fd >= 0 ? "ok" : strerror(errno));
    if (fd >= 0) close(fd);
    fd = openat(dirfd, rel, O_RDWR);
    printf(", \"openat_rel\": \"%s\"}", fd >= 0 ? "ok" : strerror(errno));
    if (fd >= 0) close(fd);
  }
  printf("}}\n");
  return 0;
}
