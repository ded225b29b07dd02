// Time open("/dev/kfd") in a fresh process (the KFD process-creation path, kfd_create_process).
// argv[1] == "hold": keep it open for argv[2] ms before exiting.
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
static double now_ms(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec * 1e3 + t.tv_nsec / 1e6; }
int main(int argc, char **argv) {
  double t0 = now_ms();
  int fd = open("/dev/kfd", O_RDWR | O_CLOEXEC);
  double t1 = now_ms();
  if (fd < 0) { perror("open /dev/kfd"); return 1; }
  if (argc > 2 && strcmp(argv[1], "hold") == 0) usleep(atoi(argv[2]) * 1000);
  printf("{\"open_ms\": %.3f, \"t_open_end\": %.3f}\n", t1 - t0, t1);
  fflush(stdout);
  close(fd);
  return 0;
}
