// amdkube-logpump: the log half of a container shim (what conmon / the containerd shim do for
// a CRI runtime): it owns the read ends of a container's stdout and stderr pipes and appends
// every line to the container's log file in the CRI log format the kubelet reads
// (pkg/kubelet/kuberuntime/logs/logs.go parseCRILog):
//
//   <RFC3339Nano UTC timestamp> <stdout|stderr> <F|P> <content>\n
//
//   F  the content is a whole line (its newline is the record's);
//   P  a partial line: a line longer than 16 KiB is cut into P records followed by the F record
//      that ends it, and output that ends without a newline is flushed as a final P record, so
//      the reader gives back exactly the bytes the container wrote.
//
//   amdkube-logpump --log PATH [--stdout-fd N] [--stderr-fd M]
//
// It runs in a session of its own, outside the container and independent of the runtime
// process: a runtime restart does not interrupt it, and it exits once every writer of both
// pipes is gone. Each record is one write(2) on an O_APPEND descriptor, made as soon as the
// bytes arrive, so `kubectl logs -f` follows the container without buffering delay.
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace {

constexpr size_t kMaxLine = 16 * 1024;   // containerd's default max container log line size
constexpr size_t kReadSize = 64 * 1024;

struct Stream {
  int fd;
  const char* name;
  std::string buf;
};

// Go's time.RFC3339Nano in UTC: trailing zeros of the fraction are dropped (and the dot with
// them when the fraction is zero).
std::string stamp() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  tm t;
  gmtime_r(&ts.tv_sec, &t);
  char b[48];
  size_t n = strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%S", &t);
  std::string s(b, n);
  if (ts.tv_nsec != 0) {
    char f[16];
    std::snprintf(f, sizeof f, ".%09ld", static_cast<long>(ts.tv_nsec));
    std::string frac(f);
    while (frac.back() == '0') frac.pop_back();
    s += frac;
  }
  s += 'Z';
  return s;
}

bool write_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t w = write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

void emit(int out, const std::string& ts, const Stream& s, char tag, const char* p, size_t n) {
  std::string rec;
  rec.reserve(ts.size() + n + 12);
  rec += ts;
  rec += ' ';
  rec += s.name;
  rec += ' ';
  rec += tag;
  rec += ' ';
  rec.append(p, n);
  rec += '\n';
  if (!write_all(out, rec.data(), rec.size())) std::perror("amdkube-logpump: write");
}

// Write out every complete line of s.buf (over-long ones as P chunks + F), the over-long head
// of an unfinished line, and — at EOF — whatever is left as a final P record.
void drain(int out, Stream& s, const std::string& ts, bool eof) {
  size_t start = 0;
  for (;;) {
    size_t nl = s.buf.find('\n', start);
    if (nl == std::string::npos) break;
    size_t len = nl - start;
    while (len > kMaxLine) {
      emit(out, ts, s, 'P', s.buf.data() + start, kMaxLine);
      start += kMaxLine;
      len -= kMaxLine;
    }
    emit(out, ts, s, 'F', s.buf.data() + start, len);
    start = nl + 1;
  }
  while (s.buf.size() - start >= kMaxLine) {
    emit(out, ts, s, 'P', s.buf.data() + start, kMaxLine);
    start += kMaxLine;
  }
  if (eof && start < s.buf.size()) {
    emit(out, ts, s, 'P', s.buf.data() + start, s.buf.size() - start);
    start = s.buf.size();
  }
  s.buf.erase(0, start);
}

int usage() {
  std::fprintf(stderr, "usage: amdkube-logpump --log PATH [--stdout-fd N] [--stderr-fd M]\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  const char* path = nullptr;
  Stream streams[2] = {{-1, "stdout", {}}, {-1, "stderr", {}}};
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--log" && i + 1 < argc) path = argv[++i];
    else if (a == "--stdout-fd" && i + 1 < argc) streams[0].fd = std::atoi(argv[++i]);
    else if (a == "--stderr-fd" && i + 1 < argc) streams[1].fd = std::atoi(argv[++i]);
    else return usage();
  }
  if (path == nullptr || (streams[0].fd < 0 && streams[1].fd < 0)) return usage();
  signal(SIGPIPE, SIG_IGN);
  int out = open(path, O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0640);
  if (out < 0) {
    std::perror("amdkube-logpump: open log");
    return 1;
  }
  for (auto& s : streams)
    if (s.fd >= 0) fcntl(s.fd, F_SETFD, FD_CLOEXEC);
  std::string chunk(kReadSize, '\0');
  for (;;) {
    pollfd pf[2];
    int idx[2];
    int n = 0;
    for (int k = 0; k < 2; ++k) {
      if (streams[k].fd < 0) continue;
      pf[n] = {streams[k].fd, POLLIN, 0};
      idx[n++] = k;
    }
    if (n == 0) break;
    int r = poll(pf, n, -1);
    if (r < 0) {
      if (errno == EINTR) continue;
      std::perror("amdkube-logpump: poll");
      break;
    }
    for (int j = 0; j < n; ++j) {
      if (!(pf[j].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      Stream& s = streams[idx[j]];
      ssize_t got = read(s.fd, &chunk[0], chunk.size());
      if (got < 0 && (errno == EINTR || errno == EAGAIN)) continue;
      std::string ts = stamp();
      if (got <= 0) {
        drain(out, s, ts, true);
        close(s.fd);
        s.fd = -1;
        continue;
      }
      s.buf.append(chunk.data(), static_cast<size_t>(got));
      drain(out, s, ts, false);
    }
  }
  for (auto& s : streams)
    if (!s.buf.empty()) drain(out, s, stamp(), true);
  close(out);
  return 0;
}
