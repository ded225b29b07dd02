// pause: the sandbox holder process of an amdkube pod (rocshim runtime).
//
// Same contract as the reference's infra container (build/pause/pause.c:17-51): sleep
// forever, reap zombies, exit 0 on SIGINT/SIGTERM. Additionally, because rocshim runs pods
// as process trees rather than inside a PID namespace when it is unprivileged, pause makes
// itself a child subreaper (PR_SET_CHILD_SUBREAPER) so orphaned descendants of the pod's
// containers are re-parented to — and reaped by — the pod's own sandbox, and it can write
// its pid to a file for the runtime's checkpoint (`pause --pidfile PATH`).
#include <signal.h>
#include <sys/prctl.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static void on_term(int sig) {
  (void)sig;
  _exit(0);
}

static void on_child(int sig) {
  (void)sig;
  int saved = errno;
  while (waitpid(-1, nullptr, WNOHANG) > 0) {
  }
  errno = saved;
}

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    if (std::strcmp(argv[i], "-v") == 0 || std::strcmp(argv[i], "--version") == 0) {
      std::printf("pause (amdkube) 3.1\n");
      return 0;
    }
    if (std::strcmp(argv[i], "--pidfile") == 0 && i + 1 < argc) {
      FILE* f = std::fopen(argv[++i], "w");
      if (f) {
        std::fprintf(f, "%d\n", static_cast<int>(getpid()));
        std::fclose(f);
      }
    }
  }
  if (getpid() != 1) {
    prctl(PR_SET_CHILD_SUBREAPER, 1, 0, 0, 0);
  }
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_term;
  if (sigaction(SIGINT, &sa, nullptr) < 0) return 1;
  if (sigaction(SIGTERM, &sa, nullptr) < 0) return 2;
  sa.sa_handler = on_child;
  sa.sa_flags = SA_NOCLDSTOP | SA_RESTART;
  if (sigaction(SIGCHLD, &sa, nullptr) < 0) return 3;
  for (;;) pause();
  return 42;
}
