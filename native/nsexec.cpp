// amdkube-nsexec: rocshim's privileged container launcher (the OCI-runtime-hook analogue).
//
// The reference hands GPU containers to the `nvidia` OCI runtime through the Docker hooks
// service (pkg/kubelet/dockershim/docker_hooks.go) which injects /dev/nvidia*. On MI355X
// the devices are /dev/kfd (one node for all compute) plus one DRM render node per GPU, so
// isolation = "the container's /dev/dri contains only its own render nodes":
//
//   amdkube-nsexec [--dev-root /dev] [--keep /dev/dri/renderD128 ...] [--hide-kfd]
//                  [--cgroup /sys/fs/cgroup/amdkube/<pod>/<ctr>] [--memory-max BYTES] [--cpuset 0-3,8]
//                  [--cpu-max "QUOTA PERIOD"] [--cgroup-wait-fd N] -- argv...
//
//  0. --cgroup-wait-fd N: block until the runtime has placed this process in its cgroup
//     (systemd driver: a transient scope made with this pid) and writes one byte to fd N;
//  1. join (creating) a cgroup-v2 leaf and apply memory.max / cpu.max / cpu.weight
//     (--cpu-weight, from the kubelet's cpu shares) and the OOM score (--oom-score-adj, QoS);
//  2. unshare a private mount namespace;
//  3. open every kept device node with O_PATH (inside the new namespace), mount a fresh tmpfs over <dev-root>/dri and
//     bind the kept nodes back from /proc/self/fd (no CAP_MKNOD needed);
//  4. --hide-kfd: bind /dev/null over <dev-root>/kfd for containers without GPUs;
//     --bind SRC:DST[:ro]: bind-mount a volume (or the pod's resolv.conf) at DST, creating an
//     empty file/directory mount point when DST is missing;
//  5. --seccomp PROFILE.json: compile the Docker-format profile to BPF (seccomp_bpf.h) and
//     install it with no_new_privs, right before exec;
//  6. --apparmor NAME: request the AppArmor profile transition on exec (`exec NAME` into
//     /proc/self/attr/apparmor/exec, or the pre-5.x /proc/self/attr/exec);
//  7. exec the container's argv.
// Pod namespaces (rocshim pod networking, applied first, in both modes):
//   --unshare net,ipc,uts   the pod sandbox (pause) gets fresh network/IPC/UTS namespaces;
//   --hostname NAME         the pod's hostname in its new UTS namespace;
//   --join net:PATH ...     a container joins its sandbox's namespaces (/proc/<pause>/ns/<type>);
//                           with --no-namespaces, user:/mnt: joins enter a running container
//                           (exec), in the order given;
//   --sysctl KEY=VALUE      namespaced sysctls (net.*, kernel.shm*, ...) written after the
//                           namespaces are set up, so they apply to the pod, never the host.
// `--no-namespaces` skips steps 1-4 (unprivileged `env` isolation still gets seccomp/AppArmor).
// Device guards (devguard.h), enforced by the kernel whatever the container does with its env:
//   --landlock        Landlock ruleset: only the --keep render nodes (and /dev/kfd unless
//                     --hide-kfd) are openable among <dev-root>/dri/* and kfd; mknod of any
//                     device node is refused. Works unprivileged (the GPU box has no userns);
//                     in namespace modes it is layered under the private /dev/dri.
//   --device-cgroup   root: attach a cgroup-v2 BPF device filter (char 226:* only the kept
//                     minors; kfd only for GPU containers) to the container's --cgroup leaf.
//   --userns          not root: a user namespace (uid/gid -> 0) owns the mount namespace, so
//                     the private /dev/dri works without privileges where userns is enabled.
// Image root filesystems (namespace modes):
//   --rootfs DIR --rootfs-upper DIR [--workdir PATH] [--user UID[:GID]]
//                     overlay the image's unpacked rootfs (lower, read-only) with the
//                     container's writable layer (upper), give it /proc, a read-only /sys, a
//                     fresh /dev (null, zero, full, random, urandom, tty, shm, the kept GPU
//                     nodes and kfd for GPU containers), bind the volumes under it, then
//                     pivot_root into it (docker_container.go:88-172 builds the container
//                     from its image the same way through dockerd/runc).
//   --caps LIST|all   capability bounding set kept for the container (comma list of names,
//                     default: the Docker default set); everything else is dropped, and
//                     no_new_privs is set, before exec.
// Any isolation step that fails is fatal (exit 126): a container never silently runs with
// more devices, or fewer syscall restrictions, than it was given.
#include <fcntl.h>
#include <sched.h>
#include <grp.h>
#include <sys/mount.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <linux/capability.h>
#include <sys/prctl.h>
#include <sys/syscall.h>

#include "devguard.h"
#include "seccomp_bpf.h"

static int die(const char* what) {
  std::fprintf(stderr, "amdkube-nsexec: %s: %s\n", what, std::strerror(errno));
  return 126;
}

static bool write_file(const std::string& path, const std::string& val) {
  int fd = open(path.c_str(), O_WRONLY | O_CLOEXEC);
  if (fd < 0) return false;
  bool ok = write(fd, val.data(), val.size()) == static_cast<ssize_t>(val.size());
  close(fd);
  return ok;
}

// AppArmor change_onexec without libapparmor: the transition happens at the next execve, so
// the container's own binary is the first thing that runs confined.
// Some kernels accept the write with no LSM behind it, so the module must report enabled first.
static bool apparmor_onexec(const std::string& profile) {
  std::ifstream en("/sys/module/apparmor/parameters/enabled");
  char c = 0;
  if (!(en >> c) || c != 'Y') {
    errno = ENOSYS;
    return false;
  }
  std::string cmd = "exec " + profile;
  return write_file("/proc/self/attr/apparmor/exec", cmd) || write_file("/proc/self/attr/exec", cmd);
}

// "0-3,8,10-11" → affinity mask (the CPU manager's exclusive or shared-pool cpuset)
static bool parse_cpuset(const std::string& spec, cpu_set_t* set) {
  CPU_ZERO(set);
  std::stringstream ss(spec);
  std::string part;
  int n = 0;
  while (std::getline(ss, part, ',')) {
    if (part.empty()) continue;
    size_t dash = part.find('-');
    char* end = nullptr;
    long lo = std::strtol(part.c_str(), &end, 10), hi = lo;
    if (dash != std::string::npos) hi = std::strtol(part.c_str() + dash + 1, &end, 10);
    if (lo < 0 || hi < lo || hi >= CPU_SETSIZE) return false;
    for (long c = lo; c <= hi; ++c) { CPU_SET(c, set); ++n; }
  }
  return n > 0;
}

static int mkdir_p(const std::string& p) {
  std::string cur;
  for (size_t i = 0; i < p.size(); ++i) {
    cur += p[i];
    if ((p[i] == '/' && i > 0) || i + 1 == p.size()) {
      if (mkdir(cur.c_str(), 0755) < 0 && errno != EEXIST) return -1;
    }
  }
  return 0;
}

static int bind_path(const std::string& src, const std::string& dst, bool ro = false) {
  struct stat ss, ds;
  if (stat(src.c_str(), &ss) < 0) return die(("bind source " + src).c_str());
  if (stat(dst.c_str(), &ds) < 0) {
    size_t slash = dst.rfind('/');
    if (slash != std::string::npos && slash > 0 && mkdir_p(dst.substr(0, slash)) < 0) return die(("mount point parent " + dst).c_str());
    if (S_ISDIR(ss.st_mode)) {
      if (mkdir(dst.c_str(), 0755) < 0 && errno != EEXIST) return die(("mount point " + dst).c_str());
    } else {
      int tfd = open(dst.c_str(), O_CREAT | O_WRONLY | O_CLOEXEC, 0644);
      if (tfd < 0) return die(("mount point " + dst).c_str());
      close(tfd);
    }
  }
  if (mount(src.c_str(), dst.c_str(), nullptr, MS_BIND | MS_REC, nullptr) < 0) return die(("bind " + dst).c_str());
  if (ro && mount(nullptr, dst.c_str(), nullptr, MS_BIND | MS_REMOUNT | MS_RDONLY | MS_REC, nullptr) < 0)
    return die(("remount read-only " + dst).c_str());
  return 0;
}

// Assemble the container's root (overlay of the image + writable layer, /proc, /sys, /dev, GPU
// nodes, volumes) and pivot_root into it. Runs inside the container's new mount namespace.
static int setup_rootfs(const std::string& lower, const std::string& upper, const std::string& dev_root,
                        const std::vector<std::string>& keep, bool hide_kfd, const std::vector<std::string>& binds,
                        int ll_rs, const std::string& workdir) {
  std::string merged = upper + "/merged", up = upper + "/upper", work = upper + "/work";
  for (auto* d : {&merged, &up, &work})
    if (mkdir_p(*d) < 0) return die(("create " + *d).c_str());
  std::string opts = "lowerdir=" + lower + ",upperdir=" + up + ",workdir=" + work;
  if (mount("overlay", merged.c_str(), "overlay", 0, opts.c_str()) < 0) return die("mount overlay root filesystem");
  if (mkdir_p(merged + "/proc") < 0 || mount("/proc", (merged + "/proc").c_str(), nullptr, MS_BIND | MS_REC, nullptr) < 0)
    return die("bind /proc");
  if (int rc = bind_path("/sys", merged + "/sys", true)) return rc;
  std::string dev = merged + "/dev";
  if (mkdir_p(dev) < 0 || mount("tmpfs", dev.c_str(), "tmpfs", MS_NOSUID, "mode=755,size=65536k") < 0) return die("mount /dev");
  for (const char* n : {"null", "zero", "full", "random", "urandom", "tty"}) {
    std::string src = std::string("/dev/") + n;
    struct stat st;
    if (stat(src.c_str(), &st) == 0)
      if (int rc = bind_path(src, dev + "/" + n)) return rc;
  }
  if (mkdir_p(dev + "/shm") < 0 || mount("tmpfs", (dev + "/shm").c_str(), "tmpfs", MS_NOSUID | MS_NODEV, "mode=1777,size=65536k") < 0)
    return die("mount /dev/shm");
  const char* links[][2] = {{"/proc/self/fd", "fd"}, {"/proc/self/fd/0", "stdin"}, {"/proc/self/fd/1", "stdout"},
                            {"/proc/self/fd/2", "stderr"}};
  for (auto& l : links)
    if (symlink(l[0], (dev + "/" + l[1]).c_str()) < 0 && errno != EEXIST) return die("create /dev link");
  for (auto& k : keep) {
    const char* base = std::strrchr(k.c_str(), '/');
    if (int rc = bind_path(k, dev + "/dri/" + (base ? base + 1 : k.c_str()))) return rc;
  }
  struct stat ks;
  if (!hide_kfd && stat((dev_root + "/kfd").c_str(), &ks) == 0)
    if (int rc = bind_path(dev_root + "/kfd", dev + "/kfd")) return rc;
  for (auto& b : binds) {
    size_t c1 = b.find(':');
    if (c1 == std::string::npos) {
      std::fprintf(stderr, "amdkube-nsexec: bad --bind %s\n", b.c_str());
      return 126;
    }
    std::string src = b.substr(0, c1), dst = b.substr(c1 + 1);
    bool ro = dst.size() > 3 && dst.compare(dst.size() - 3, 3, ":ro") == 0;
    if (ro) dst = dst.substr(0, dst.size() - 3);
    if (dst.empty() || dst[0] != '/' || dst.find("/../") != std::string::npos) {
      std::fprintf(stderr, "amdkube-nsexec: bad --bind destination %s\n", dst.c_str());
      return 126;
    }
    if (int rc = bind_path(src, merged + dst, ro)) return rc;
  }
  // the container's whole tree is one new mount root: grant it (the host-view rules cannot see it)
  if (ll_rs >= 0 && !amdkube_devguard::landlock_grant(ll_rs, merged)) return die("landlock grant rootfs");
  std::string old = merged + "/.amdkube-oldroot";
  if (mkdir(old.c_str(), 0700) < 0 && errno != EEXIST) return die("create old root");
  if (syscall(SYS_pivot_root, merged.c_str(), old.c_str()) < 0) return die("pivot_root");
  if (chdir("/") < 0) return die("chdir /");
  if (umount2("/.amdkube-oldroot", MNT_DETACH) < 0) return die("detach old root");
  rmdir("/.amdkube-oldroot");
  if (!workdir.empty()) {
    mkdir_p(workdir);
    if (chdir(workdir.c_str()) < 0) return die(("chdir " + workdir).c_str());
  }
  return 0;
}

static int switch_user(const std::string& spec) {
  char* end = nullptr;
  long uid = std::strtol(spec.c_str(), &end, 10);
  long gid = uid;
  if (end && *end == ':') gid = std::strtol(end + 1, &end, 10);
  if (uid < 0 || gid < 0 || (end && *end)) {
    std::fprintf(stderr, "amdkube-nsexec: --user wants UID[:GID], got %s\n", spec.c_str());
    return 126;
  }
  if (setgroups(0, nullptr) < 0 && errno != EPERM) return die("setgroups");
  if (setgid(static_cast<gid_t>(gid)) < 0) return die("setgid");
  if (setuid(static_cast<uid_t>(uid)) < 0) return die("setuid");
  return 0;
}

static int ns_flag(const std::string& t) {
  if (t == "net") return CLONE_NEWNET;
  if (t == "ipc") return CLONE_NEWIPC;
  if (t == "uts") return CLONE_NEWUTS;
  if (t == "user") return CLONE_NEWUSER;   // exec into a userns container: join its user namespace first
  if (t == "mnt") return CLONE_NEWNS;      // ... then its mount namespace (root and cwd become its root)
  return 0;
}

static int pod_namespaces(const std::vector<std::string>& joins, const std::string& unshare_list,
                          const std::string& hostname, const std::vector<std::string>& sysctls) {
  for (auto& j : joins) {   // type:path
    size_t c = j.find(':');
    int flag = c == std::string::npos ? 0 : ns_flag(j.substr(0, c));
    if (!flag) {
      std::fprintf(stderr, "amdkube-nsexec: bad --join %s\n", j.c_str());
      return 126;
    }
    int fd = open(j.substr(c + 1).c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return die(("open namespace " + j).c_str());
    if (setns(fd, flag) < 0) return die(("setns " + j).c_str());
    close(fd);
  }
  if (!unshare_list.empty()) {
    int flags = 0;
    std::stringstream ss(unshare_list);
    std::string t;
    while (std::getline(ss, t, ',')) {
      int f = ns_flag(t);
      if (!f) {
        std::fprintf(stderr, "amdkube-nsexec: bad --unshare %s\n", t.c_str());
        return 126;
      }
      flags |= f;
    }
    if (unshare(flags) < 0) return die(("unshare " + unshare_list).c_str());
  }
  if (!hostname.empty() && sethostname(hostname.data(), hostname.size()) < 0) return die("sethostname");
  for (auto& kv : sysctls) {
    size_t eq = kv.find('=');
    if (eq == std::string::npos || eq == 0 || kv.find("..") != std::string::npos || kv[0] == '/') {
      std::fprintf(stderr, "amdkube-nsexec: bad --sysctl %s\n", kv.c_str());
      return 126;
    }
    std::string key = kv.substr(0, eq);
    for (auto& ch : key) if (ch == '.') ch = '/';
    if (!write_file("/proc/sys/" + key, kv.substr(eq + 1))) return die(("sysctl " + kv.substr(0, eq)).c_str());
  }
  return 0;
}

// Docker's default capability set (the reference's containers run with it, docker/oci/defaults.go)
static const char* kDefaultCaps[] = {"chown", "dac_override", "fsetid", "fowner", "mknod", "net_raw", "setgid", "setuid",
                                     "setfcap", "setpcap", "net_bind_service", "sys_chroot", "kill", "audit_write"};
static const char* kCapNames[] = {"chown", "dac_override", "dac_read_search", "fowner", "fsetid", "kill", "setgid",
                                  "setuid", "setpcap", "linux_immutable", "net_bind_service", "net_broadcast", "net_admin",
                                  "net_raw", "ipc_lock", "ipc_owner", "sys_module", "sys_rawio", "sys_chroot", "sys_ptrace",
                                  "sys_pacct", "sys_admin", "sys_boot", "sys_nice", "sys_resource", "sys_time",
                                  "sys_tty_config", "mknod", "lease", "audit_write", "audit_control", "setfcap",
                                  "mac_override", "mac_admin", "syslog", "wake_alarm", "block_suspend", "audit_read",
                                  "perfmon", "bpf", "checkpoint_restore"};

static int cap_index(std::string n) {
  for (auto& ch : n) ch = static_cast<char>(std::tolower(ch));
  if (n.rfind("cap_", 0) == 0) n = n.substr(4);
  for (int c = 0; c < static_cast<int>(sizeof(kCapNames) / sizeof(kCapNames[0])); ++c)
    if (n == kCapNames[c]) return c;
  return -1;
}

// Keep only `spec` (comma list, "all" keeps everything) in the bounding, inheritable and ambient
// sets, then no_new_privs: an exec'd setuid binary cannot gain anything back.
static bool limit_caps(const std::string& spec, std::string* err) {
  if (spec == "all") return true;
  uint64_t keep = 0;
  std::stringstream ss(spec == "default" ? "" : spec);
  std::string t;
  if (spec == "default") {
    for (auto* n : kDefaultCaps) keep |= 1ULL << cap_index(n);
  }
  while (std::getline(ss, t, ',')) {
    if (t.empty() || t == "none") continue;
    int c = cap_index(t);
    if (c < 0) {
      *err = "unknown capability " + t;
      return false;
    }
    keep |= 1ULL << c;
  }
  prctl(PR_CAP_AMBIENT, PR_CAP_AMBIENT_CLEAR_ALL, 0, 0, 0);
  for (int c = 0; c <= 63; ++c) {
    if (keep & (1ULL << c)) continue;
    if (prctl(PR_CAPBSET_READ, c, 0, 0, 0) <= 0) continue;   // absent or not supported
    if (prctl(PR_CAPBSET_DROP, c, 0, 0, 0) < 0) {
      *err = std::string("drop capability ") + (c < 41 ? kCapNames[c] : std::to_string(c)) + ": " + std::strerror(errno);
      return false;
    }
  }
  __user_cap_header_struct hdr{_LINUX_CAPABILITY_VERSION_3, 0};
  __user_cap_data_struct data[2]{};
  if (syscall(SYS_capget, &hdr, data) == 0) {
    for (int w = 0; w < 2; ++w) {
      uint32_t k = static_cast<uint32_t>(keep >> (32 * w));
      data[w].effective &= k;
      data[w].permitted &= k;
      data[w].inheritable &= k;
    }
    if (syscall(SYS_capset, &hdr, data) < 0) {
      *err = std::string("capset: ") + std::strerror(errno);
      return false;
    }
  }
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) < 0) {
    *err = std::string("no_new_privs: ") + std::strerror(errno);
    return false;
  }
  return true;
}

// not root: a user namespace owning the mount namespace (uid/gid map to 0 inside)
static int enter_userns() {
  uid_t uid = getuid();
  gid_t gid = getgid();
  if (unshare(CLONE_NEWUSER | CLONE_NEWNS) < 0) return die("unshare(CLONE_NEWUSER|CLONE_NEWNS)");
  if (!write_file("/proc/self/setgroups", "deny")) return die("setgroups deny");
  if (!write_file("/proc/self/uid_map", "0 " + std::to_string(uid) + " 1")) return die("uid_map");
  if (!write_file("/proc/self/gid_map", "0 " + std::to_string(gid) + " 1")) return die("gid_map");
  return 0;
}

// --probe: one JSON line naming the isolation mechanisms this node offers, for rocshim's
// isolation=auto (root + cgroup v2 → namespaces; user namespaces → userns; Landlock → landlock).
static int probe() {
  int abi = amdkube_devguard::landlock_abi();
  pid_t pid = fork();
  bool userns = false;
  if (pid == 0) _exit(unshare(CLONE_NEWUSER | CLONE_NEWNS) == 0 ? 0 : 1);
  if (pid > 0) {
    int st = 0;
    waitpid(pid, &st, 0);
    userns = WIFEXITED(st) && WEXITSTATUS(st) == 0;
  }
  struct stat cs;
  bool cg2 = stat("/sys/fs/cgroup/cgroup.controllers", &cs) == 0;
  std::printf("{\"root\": %s, \"landlock_abi\": %d, \"userns\": %s, \"cgroup2\": %s, \"cgroup2_writable\": %s}\n",
              geteuid() == 0 ? "true" : "false", abi < 0 ? 0 : abi, userns ? "true" : "false", cg2 ? "true" : "false",
              cg2 && access("/sys/fs/cgroup", W_OK) == 0 ? "true" : "false");
  return 0;
}

// The devview preload (AMDKUBE_DEVVIEW_LIB) is armed for the workload only: this launcher
// enumerates the device root itself to build the Landlock ruleset, so it must see every node.
static void arm_devview() {
  const char* lib = std::getenv("AMDKUBE_DEVVIEW_LIB");
  if (!lib || !*lib) return;
  const char* pre = std::getenv("LD_PRELOAD");
  std::string v = lib;
  if (pre && *pre) v += std::string(":") + pre;
  setenv("LD_PRELOAD", v.c_str(), 1);
  unsetenv("AMDKUBE_DEVVIEW_LIB");
}

int main(int argc, char** argv) {
  if (argc == 2 && std::string(argv[1]) == "--probe") return probe();
  std::string dev_root = "/dev", cgroup, mem_max, cpu_max, cpu_weight, oom_adj;
  std::vector<std::string> keep, binds;
  bool hide_kfd = false, no_ns = false, use_landlock = false, device_cgroup = false, userns = false;
  std::string caps, rootfs, rootfs_upper, workdir, user;
  std::string seccomp_profile, apparmor, cpuset, unshare_list, hostname;
  std::vector<std::string> joins, sysctls;
  int wait_fd = -1;
  int i = 1;
  for (; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--") {
      ++i;
      break;
    } else if (a == "--dev-root" && i + 1 < argc) dev_root = argv[++i];
    else if (a == "--keep" && i + 1 < argc) keep.push_back(argv[++i]);
    else if (a == "--hide-kfd") hide_kfd = true;
    else if (a == "--bind" && i + 1 < argc) binds.push_back(argv[++i]);
    else if (a == "--cgroup" && i + 1 < argc) cgroup = argv[++i];
    else if (a == "--memory-max" && i + 1 < argc) mem_max = argv[++i];
    else if (a == "--cpu-max" && i + 1 < argc) cpu_max = argv[++i];
    else if (a == "--cpu-weight" && i + 1 < argc) cpu_weight = argv[++i];
    else if (a == "--oom-score-adj" && i + 1 < argc) oom_adj = argv[++i];
    else if (a == "--seccomp" && i + 1 < argc) seccomp_profile = argv[++i];
    else if (a == "--apparmor" && i + 1 < argc) apparmor = argv[++i];
    else if (a == "--no-namespaces") no_ns = true;
    else if (a == "--landlock") use_landlock = true;
    else if (a == "--device-cgroup") device_cgroup = true;
    else if (a == "--userns") userns = true;
    else if (a == "--caps" && i + 1 < argc) caps = argv[++i];
    else if (a == "--rootfs" && i + 1 < argc) rootfs = argv[++i];
    else if (a == "--rootfs-upper" && i + 1 < argc) rootfs_upper = argv[++i];
    else if (a == "--workdir" && i + 1 < argc) workdir = argv[++i];
    else if (a == "--user" && i + 1 < argc) user = argv[++i];
    else if (a == "--cpuset" && i + 1 < argc) cpuset = argv[++i];
    else if (a == "--unshare" && i + 1 < argc) unshare_list = argv[++i];
    else if (a == "--hostname" && i + 1 < argc) hostname = argv[++i];
    else if (a == "--join" && i + 1 < argc) joins.push_back(argv[++i]);
    else if (a == "--sysctl" && i + 1 < argc) sysctls.push_back(argv[++i]);
    else if (a == "--cgroup-wait-fd" && i + 1 < argc) wait_fd = std::atoi(argv[++i]);
    else {
      std::fprintf(stderr, "amdkube-nsexec: unknown argument %s\n", a.c_str());
      return 126;
    }
  }
  if (i >= argc) {
    std::fprintf(stderr, "usage: amdkube-nsexec [options] -- argv...\n");
    return 126;
  }
  std::vector<sock_filter> filter;
  if (!seccomp_profile.empty()) {   // compile before any change, so a bad profile fails cleanly
    std::ifstream in(seccomp_profile);
    if (!in) return die(("read seccomp profile " + seccomp_profile).c_str());
    std::stringstream ss;
    ss << in.rdbuf();
    std::string err;
    if (!amdkube_seccomp::compile(ss.str(), &filter, &err)) {
      std::fprintf(stderr, "amdkube-nsexec: seccomp profile %s: %s\n", seccomp_profile.c_str(), err.c_str());
      return 126;
    }
  }
  if (wait_fd >= 0) {
    // the runtime first places this process in its cgroup (the systemd driver: a transient
    // scope created with our pid) and then releases it: one byte = placed, EOF = failed
    char b = 0;
    ssize_t n;
    do n = read(wait_fd, &b, 1); while (n < 0 && errno == EINTR);
    close(wait_fd);
    if (n != 1) {
      std::fprintf(stderr, "amdkube-nsexec: the runtime did not place the container in its cgroup\n");
      return 126;
    }
  }
  if (!cpuset.empty()) {   // inherited by every process of the container
    cpu_set_t set;
    if (!parse_cpuset(cpuset, &set)) {
      std::fprintf(stderr, "amdkube-nsexec: bad --cpuset %s\n", cpuset.c_str());
      return 126;
    }
    if (sched_setaffinity(0, sizeof(set), &set) < 0) return die("sched_setaffinity");
  }
  if (no_ns && !cgroup.empty()) {
    // exec into a running container: join its cgroup leaf (its limits stay as they are)
    if (!write_file(cgroup + "/cgroup.procs", std::to_string(getpid()))) return die("join cgroup");
  }
  if (int rc = pod_namespaces(joins, unshare_list, hostname, sysctls)) return rc;
  if (no_ns && !workdir.empty() && chdir(workdir.c_str()) < 0) return die(("chdir " + workdir).c_str());
  if (no_ns) {
    std::string err;
    if (use_landlock) {
      // kernel-enforced device view for an unprivileged node (no mount namespace to hide nodes in)
      if (!amdkube_devguard::landlock_apply(amdkube_devguard::plan(dev_root, keep, hide_kfd), &err)) {
        std::fprintf(stderr, "amdkube-nsexec: %s\n", err.c_str());
        return 126;
      }
    }
    if (!caps.empty() && !limit_caps(caps, &err)) {
      std::fprintf(stderr, "amdkube-nsexec: %s\n", err.c_str());
      return 126;
    }
    if (!apparmor.empty() && !apparmor_onexec(apparmor)) return die(("AppArmor profile " + apparmor).c_str());
    if (!filter.empty() && !amdkube_seccomp::apply(filter, &err)) {
      std::fprintf(stderr, "amdkube-nsexec: %s\n", err.c_str());
      return 126;
    }
    arm_devview();
    execvp(argv[i], argv + i);
    return die(("exec " + std::string(argv[i])).c_str());
  }
  if (!cgroup.empty()) {
    if (mkdir_p(cgroup) < 0) return die("create cgroup");
    if (!mem_max.empty()) write_file(cgroup + "/memory.max", mem_max);
    if (!cpu_max.empty()) write_file(cgroup + "/cpu.max", cpu_max);
    if (!cpu_weight.empty()) write_file(cgroup + "/cpu.weight", cpu_weight);
    if (!cpuset.empty()) write_file(cgroup + "/cpuset.cpus", cpuset);   // when the cpuset controller is delegated
    if (!write_file(cgroup + "/cgroup.procs", std::to_string(getpid()))) return die("join cgroup");
    if (device_cgroup) {
      std::string err;
      if (!amdkube_devguard::cgroup_device_filter(cgroup, keep, dev_root, hide_kfd, &err)) {
        std::fprintf(stderr, "amdkube-nsexec: %s\n", err.c_str());
        return 126;
      }
    }
  }
  // lowering the score needs CAP_SYS_RESOURCE, which the privileged launcher has
  if (!oom_adj.empty() && !write_file("/proc/self/oom_score_adj", oom_adj)) return die("oom_score_adj");
  // the Landlock plan is taken on the host view (rules bind to the real inodes: the kept nodes
  // stay reachable through their bind mounts, the real kfd stays denied behind the /dev/null bind)
  int ll_rs = -1;
  if (use_landlock) {
    std::string err;
    ll_rs = amdkube_devguard::landlock_ruleset(amdkube_devguard::plan(dev_root, keep, hide_kfd), &err);
    if (ll_rs < 0) {
      std::fprintf(stderr, "amdkube-nsexec: %s\n", err.c_str());
      return 126;
    }
  }
  if (userns && getuid() != 0) {
    if (int rc = enter_userns()) return rc;
  } else if (unshare(CLONE_NEWNS) < 0) {
    return die("unshare(CLONE_NEWNS)");
  }
  if (mount(nullptr, "/", nullptr, MS_REC | MS_PRIVATE, nullptr) < 0) return die("make / rprivate");
  if (!rootfs.empty()) {
    if (rootfs_upper.empty()) {
      std::fprintf(stderr, "amdkube-nsexec: --rootfs needs --rootfs-upper\n");
      return 126;
    }
    if (int rc = setup_rootfs(rootfs, rootfs_upper, dev_root, keep, hide_kfd, binds, ll_rs, workdir)) return rc;
    binds.clear();
    keep.clear();
    hide_kfd = false;
  }
  // open the kept nodes inside the new namespace (a bind source must belong to it)
  std::vector<int> fds;
  for (auto& k : keep) {
    int fd = open(k.c_str(), O_PATH | O_CLOEXEC);
    if (fd < 0) return die(("open kept device " + k).c_str());
    fds.push_back(fd);
  }
  std::string dri = dev_root + "/dri";
  struct stat st;
  if (rootfs.empty() && stat(dri.c_str(), &st) == 0) {
    if (mount("tmpfs", dri.c_str(), "tmpfs", MS_NOSUID | MS_NOEXEC, "mode=755,size=64k") < 0) return die("mount tmpfs on dri");
    for (size_t k = 0; k < keep.size(); ++k) {
      const char* base = std::strrchr(keep[k].c_str(), '/');
      std::string target = dri + "/" + (base ? base + 1 : keep[k].c_str());
      int tfd = open(target.c_str(), O_CREAT | O_WRONLY | O_CLOEXEC, 0666);
      if (tfd < 0) return die(("create mount point " + target).c_str());
      close(tfd);
      std::string src = "/proc/self/fd/" + std::to_string(fds[k]);
      if (mount(src.c_str(), target.c_str(), nullptr, MS_BIND, nullptr) < 0) return die(("bind " + target).c_str());
    }
  }
  if (hide_kfd) {
    std::string kfd = dev_root + "/kfd";
    if (stat(kfd.c_str(), &st) == 0 && mount("/dev/null", kfd.c_str(), nullptr, MS_BIND, nullptr) < 0) return die("hide kfd");
  }
  for (int fd : fds) close(fd);
  for (auto& b : binds) {
    size_t c1 = b.find(':');
    if (c1 == std::string::npos) {
      std::fprintf(stderr, "amdkube-nsexec: bad --bind %s\n", b.c_str());
      return 126;
    }
    std::string src = b.substr(0, c1), rest = b.substr(c1 + 1), dst = rest;
    bool ro = false;
    if (rest.size() > 3 && rest.compare(rest.size() - 3, 3, ":ro") == 0) {
      dst = rest.substr(0, rest.size() - 3);
      ro = true;
    }
    struct stat ss, ds;
    if (stat(src.c_str(), &ss) < 0) return die(("bind source " + src).c_str());
    if (stat(dst.c_str(), &ds) < 0) {
      size_t slash = dst.rfind('/');
      if (slash != std::string::npos && slash > 0 && mkdir_p(dst.substr(0, slash)) < 0) return die(("mount point parent " + dst).c_str());
      if (S_ISDIR(ss.st_mode)) {
        if (mkdir(dst.c_str(), 0755) < 0 && errno != EEXIST) return die(("mount point " + dst).c_str());
      } else {
        int tfd = open(dst.c_str(), O_CREAT | O_WRONLY | O_CLOEXEC, 0644);
        if (tfd < 0) return die(("mount point " + dst).c_str());
        close(tfd);
      }
    }
    if (mount(src.c_str(), dst.c_str(), nullptr, MS_BIND | MS_REC, nullptr) < 0) return die(("bind " + dst).c_str());
    if (ro && mount(nullptr, dst.c_str(), nullptr, MS_BIND | MS_REMOUNT | MS_RDONLY | MS_REC, nullptr) < 0)
      return die(("remount read-only " + dst).c_str());
    // a new mount point is not beneath any granted inode: grant the volume itself
    if (ll_rs >= 0 && !amdkube_devguard::landlock_grant(ll_rs, dst)) return die(("landlock grant " + dst).c_str());
  }
  {
    std::string err;
    // after the mounts: a Landlock-restricted process may not change its mount topology, so the
    // container cannot unmount the private /dev/dri either
    if (ll_rs >= 0 && !amdkube_devguard::landlock_restrict(ll_rs, &err)) {
      std::fprintf(stderr, "amdkube-nsexec: %s\n", err.c_str());
      return 126;
    }
    if (!limit_caps(caps.empty() ? "default" : caps, &err)) {
      std::fprintf(stderr, "amdkube-nsexec: %s\n", err.c_str());
      return 126;
    }
  }
  if (!user.empty())
    if (int rc = switch_user(user)) return rc;
  if (!apparmor.empty() && !apparmor_onexec(apparmor)) return die(("AppArmor profile " + apparmor).c_str());
  if (!filter.empty()) {
    std::string err;
    if (!amdkube_seccomp::apply(filter, &err)) {
      std::fprintf(stderr, "amdkube-nsexec: %s\n", err.c_str());
      return 126;
    }
  }
  arm_devview();
  execvp(argv[i], argv + i);
  return die(("exec " + std::string(argv[i])).c_str());
}
