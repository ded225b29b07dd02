// devguard.h — GPU device isolation that does not need root (Landlock) and the cgroup-v2 device
// filter used when it does (BPF_PROG_TYPE_CGROUP_DEVICE).
//
// The reference hands the container's device list to Docker (HostConfig.Resources.Devices,
// pkg/kubelet/dockershim/docker_container.go:155-172, from makeDevices in
// pkg/kubelet/kuberuntime/kuberuntime_container.go:277) and runc enforces it with the devices
// cgroup. An MI355X node exposes one /dev/kfd for all compute plus one DRM render node per GPU,
// so a container's device view is "kfd iff it has GPUs, and only its own render nodes".
//
// Landlock (unprivileged, inherited across exec, never removable):
//   handled rights = READ_FILE | WRITE_FILE | MAKE_CHAR | MAKE_BLOCK. Rules grant READ|WRITE on
//   every file hierarchy EXCEPT the denied device nodes: for each directory on the path from "/"
//   to a denied node we grant each child that is neither denied nor itself on such a path.
//   MAKE_CHAR / MAKE_BLOCK are granted nowhere, so mknod of any device node fails. Rules bind to
//   inodes, so /proc/<pid>/root/dev/dri/renderDX, symlinks and /proc/<pid>/fd re-opens resolve
//   to the same denied inode. Other mounts of the same device filesystem (a second devtmpfs
//   mount, a single bind-mounted node) are found in /proc/self/mountinfo and denied too.
//   Limitation: a node for the same major:minor that root created with mknod on some other
//   filesystem is not seen; the cgroup device filter (root only) covers that case.
//
// Cgroup device filter (root, cgroup v2): a BPF program attached to the container's leaf that
// rejects char 226:* (DRM) except the kept minors, and the kfd node unless the container has a
// GPU. Everything else stays allowed, as for the container's other devices.
#pragma once

#include <dirent.h>
#include <fcntl.h>
#include <linux/bpf.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/sysmacros.h>
#include <unistd.h>

#include <cerrno>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <set>
#include <sstream>
#include <string>
#include <vector>

namespace amdkube_devguard {

// uapi/linux/landlock.h (defined here so an older header does not limit the build)
constexpr uint64_t kReadFile = 1ULL << 2, kWriteFile = 1ULL << 1, kMakeChar = 1ULL << 6, kMakeBlock = 1ULL << 11;
constexpr int kRulePathBeneath = 1;
struct RulesetAttr {
  uint64_t handled_access_fs;
};
struct PathBeneathAttr {
  uint64_t allowed_access;
  int32_t parent_fd;
} __attribute__((packed));

inline int landlock_abi() {
  long v = syscall(SYS_landlock_create_ruleset, nullptr, 0, 1U /* LANDLOCK_CREATE_RULESET_VERSION */);
  return v < 0 ? -errno : static_cast<int>(v);
}

inline std::string real(const std::string& p) {
  char buf[PATH_MAX];
  return realpath(p.c_str(), buf) ? std::string(buf) : p;
}

inline std::string parent_of(const std::string& p) {
  size_t s = p.rfind('/');
  return s == 0 || s == std::string::npos ? "/" : p.substr(0, s);
}

struct Mount {
  unsigned major = 0, minor = 0;
  std::string root, point;
};

inline std::string unescape_mount(const std::string& s) {   // mountinfo octal escapes (\040 = space)
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '\\' && i + 3 < s.size()) {
      o += static_cast<char>(std::strtol(s.substr(i + 1, 3).c_str(), nullptr, 8));
      i += 3;
    } else {
      o += s[i];
    }
  }
  return o;
}

inline std::vector<Mount> mountinfo() {
  std::vector<Mount> out;
  std::ifstream in("/proc/self/mountinfo");
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string id, parent, mm, root, point;
    if (!(ss >> id >> parent >> mm >> root >> point)) continue;
    Mount m;
    if (std::sscanf(mm.c_str(), "%u:%u", &m.major, &m.minor) != 2) continue;
    m.root = unescape_mount(root);
    m.point = unescape_mount(point);
    out.push_back(m);
  }
  return out;
}

// Every path by which the file at `p` is reachable through a mount of its filesystem.
inline std::vector<std::string> aliases(const std::string& p, const std::vector<Mount>& mounts) {
  std::vector<std::string> out;
  struct stat st;
  if (lstat(p.c_str(), &st) < 0) return out;
  // the mount p is reached through: longest mount point that prefixes it, on p's device
  const Mount* own = nullptr;
  for (auto& m : mounts) {
    if (makedev(m.major, m.minor) != st.st_dev) continue;
    bool prefix = m.point == "/" || p == m.point || p.compare(0, m.point.size() + 1, m.point + "/") == 0;
    if (prefix && (!own || m.point.size() > own->point.size())) own = &m;
  }
  if (!own) return out;
  std::string tail = p == own->point ? "" : p.substr(own->point == "/" ? 0 : own->point.size());
  std::string fsrel = (own->root == "/" ? "" : own->root) + tail;   // path inside the filesystem
  if (fsrel.empty()) fsrel = "/";
  for (auto& m : mounts) {
    if (makedev(m.major, m.minor) != st.st_dev || &m == own) continue;
    std::string r = m.root == "/" ? "" : m.root;
    if (fsrel == m.root || fsrel.compare(0, r.size() + 1, r + "/") == 0) {
      std::string rest = fsrel.substr(r.size());
      std::string a = (m.point == "/" ? "" : m.point) + rest;
      if (a.empty()) a = "/";
      if (a != p) out.push_back(a);
    }
  }
  return out;
}

struct Plan {
  std::set<std::string> deny;          // device nodes (and aliases) the container must not open
  std::vector<std::string> grant;      // hierarchies granted READ|WRITE
};

// Decide which nodes to deny: every entry of <dev_root>/dri that is not kept, and <dev_root>/kfd
// when the container has no GPU; then the grant set that covers everything else.
inline Plan plan(const std::string& dev_root, const std::vector<std::string>& keep, bool hide_kfd) {
  Plan pl;
  std::string root = real(dev_root);
  std::set<std::string> kept;
  for (auto& k : keep) kept.insert(real(k));
  std::string dri = root + "/dri";
  if (DIR* d = opendir(dri.c_str())) {
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n == "." || n == "..") continue;
      std::string p = dri + "/" + n;
      struct stat st;
      if (lstat(p.c_str(), &st) < 0 || S_ISLNK(st.st_mode) || S_ISDIR(st.st_mode)) continue;   // by-path/ holds links
      if (!kept.count(p)) pl.deny.insert(p);
    }
    closedir(d);
  }
  struct stat st;
  if (hide_kfd && lstat((root + "/kfd").c_str(), &st) == 0) pl.deny.insert(root + "/kfd");
  auto mounts = mountinfo();
  std::set<std::string> extra;
  for (auto& p : pl.deny)
    for (auto& a : aliases(p, mounts)) extra.insert(a);
  // an alias of a kept node is fine; an alias that is itself kept must stay reachable
  for (auto& a : extra)
    if (!kept.count(a)) pl.deny.insert(a);
  if (pl.deny.empty()) {
    pl.grant.push_back("/");
    return pl;
  }
  std::set<std::string> chain;   // directories on a path from "/" to a denied node
  for (auto& p : pl.deny) {
    std::string c = parent_of(p);
    while (true) {
      chain.insert(c);
      if (c == "/") break;
      c = parent_of(c);
    }
  }
  for (auto& c : chain) {
    DIR* d = opendir(c.c_str());
    if (!d) continue;   // unreadable: nothing below it is granted (stricter, never looser)
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n == "." || n == "..") continue;
      std::string p = (c == "/" ? "" : c) + "/" + n;
      if (chain.count(p) || pl.deny.count(p)) continue;
      struct stat es;
      if (lstat(p.c_str(), &es) < 0 || S_ISLNK(es.st_mode)) continue;   // a link resolves to its target
      pl.grant.push_back(p);
    }
    closedir(d);
  }
  return pl;
}

// Build the ruleset for a plan (not yet enforced): returns the ruleset fd, or -1 with *err set.
inline int landlock_ruleset(const Plan& pl, std::string* err, int* nrules = nullptr) {
  int abi = landlock_abi();
  if (abi < 1) {
    *err = std::string("Landlock unavailable: ") + std::strerror(-abi);
    return -1;
  }
  RulesetAttr attr{kReadFile | kWriteFile | kMakeChar | kMakeBlock};
  int rs = static_cast<int>(syscall(SYS_landlock_create_ruleset, &attr, sizeof(attr), 0));
  if (rs < 0) {
    *err = std::string("landlock_create_ruleset: ") + std::strerror(errno);
    return -1;
  }
  fcntl(rs, F_SETFD, FD_CLOEXEC);
  int n = 0;
  for (auto& g : pl.grant) {
    int fd = open(g.c_str(), O_PATH | O_CLOEXEC | O_NOFOLLOW);
    if (fd < 0) continue;
    PathBeneathAttr pb{kReadFile | kWriteFile, fd};
    if (syscall(SYS_landlock_add_rule, rs, kRulePathBeneath, &pb, 0) == 0) ++n;
    close(fd);
  }
  if (nrules) *nrules = n;
  return rs;
}

// Grant one more hierarchy (a volume bind-mounted at a new mount point after the plan was taken).
inline bool landlock_grant(int rs, const std::string& path) {
  int fd = open(path.c_str(), O_PATH | O_CLOEXEC);
  if (fd < 0) return false;
  PathBeneathAttr pb{kReadFile | kWriteFile, fd};
  bool ok = syscall(SYS_landlock_add_rule, rs, kRulePathBeneath, &pb, 0) == 0;
  close(fd);
  return ok;
}

// Enforce on this process and everything it execs (sets no_new_privs). Consumes rs.
inline bool landlock_restrict(int rs, std::string* err) {
  bool ok = true;
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) < 0) {
    *err = std::string("no_new_privs: ") + std::strerror(errno);
    ok = false;
  } else if (syscall(SYS_landlock_restrict_self, rs, 0) < 0) {
    *err = std::string("landlock_restrict_self: ") + std::strerror(errno);
    ok = false;
  }
  close(rs);
  return ok;
}

inline bool landlock_apply(const Plan& pl, std::string* err) {
  int rs = landlock_ruleset(pl, err);
  return rs >= 0 && landlock_restrict(rs, err);
}

// ---------------------------------------------------------------- cgroup-v2 device filter (root)
struct DevRule {
  uint32_t major, minor;
};

// BPF program: allow unless (char && major==226 && minor not kept) or (char && kfd && !gpu).
inline std::vector<bpf_insn> device_program(const std::vector<uint32_t>& kept_minors, bool has_kfd, DevRule kfd, bool allow_kfd) {
  std::vector<bpf_insn> p;
  auto ins = [&](uint8_t code, uint8_t dst, uint8_t src, int16_t off, int32_t imm) {
    bpf_insn i{};
    i.code = code;
    i.dst_reg = dst;
    i.src_reg = src;
    i.off = off;
    i.imm = imm;
    p.push_back(i);
  };
  // r2 = ctx->access_type & 0xffff (device type), r3 = major, r4 = minor
  ins(BPF_LDX | BPF_W | BPF_MEM, BPF_REG_2, BPF_REG_1, 0, 0);
  ins(BPF_ALU64 | BPF_AND | BPF_K, BPF_REG_2, 0, 0, 0xffff);
  ins(BPF_LDX | BPF_W | BPF_MEM, BPF_REG_3, BPF_REG_1, 4, 0);
  ins(BPF_LDX | BPF_W | BPF_MEM, BPF_REG_4, BPF_REG_1, 8, 0);
  // not a char device → allow
  size_t jchar = p.size();
  ins(BPF_JMP | BPF_JNE | BPF_K, BPF_REG_2, 0, 0 /*patched*/, BPF_DEVCG_DEV_CHAR);
  // kfd
  if (has_kfd) {
    ins(BPF_JMP | BPF_JNE | BPF_K, BPF_REG_3, 0, 3, static_cast<int32_t>(kfd.major));
    ins(BPF_JMP | BPF_JNE | BPF_K, BPF_REG_4, 0, 2, static_cast<int32_t>(kfd.minor));
    ins(BPF_ALU64 | BPF_MOV | BPF_K, BPF_REG_0, 0, 0, allow_kfd ? 1 : 0);
    ins(BPF_JMP | BPF_EXIT, 0, 0, 0, 0);
  }
  // DRM major 226: allow only kept minors
  size_t jdrm = p.size();
  ins(BPF_JMP | BPF_JNE | BPF_K, BPF_REG_3, 0, 0 /*patched*/, 226);
  for (uint32_t m : kept_minors) {
    ins(BPF_JMP | BPF_JNE | BPF_K, BPF_REG_4, 0, 2, static_cast<int32_t>(m));
    ins(BPF_ALU64 | BPF_MOV | BPF_K, BPF_REG_0, 0, 0, 1);
    ins(BPF_JMP | BPF_EXIT, 0, 0, 0, 0);
  }
  ins(BPF_ALU64 | BPF_MOV | BPF_K, BPF_REG_0, 0, 0, 0);
  ins(BPF_JMP | BPF_EXIT, 0, 0, 0, 0);
  size_t allow = p.size();
  ins(BPF_ALU64 | BPF_MOV | BPF_K, BPF_REG_0, 0, 0, 1);
  ins(BPF_JMP | BPF_EXIT, 0, 0, 0, 0);
  p[jchar].off = static_cast<int16_t>(allow - jchar - 1);
  p[jdrm].off = static_cast<int16_t>(allow - jdrm - 1);
  return p;
}

inline bool cgroup_device_filter(const std::string& cgroup_dir, const std::vector<std::string>& keep,
                                 const std::string& dev_root, bool hide_kfd, std::string* err) {
  std::vector<uint32_t> minors;
  for (auto& k : keep) {
    struct stat st;
    if (stat(k.c_str(), &st) == 0 && S_ISCHR(st.st_mode) && major(st.st_rdev) == 226) minors.push_back(minor(st.st_rdev));
  }
  struct stat ks;
  bool has_kfd = stat((dev_root + "/kfd").c_str(), &ks) == 0 && S_ISCHR(ks.st_mode);
  DevRule kfd{has_kfd ? major(ks.st_rdev) : 0, has_kfd ? minor(ks.st_rdev) : 0};
  auto prog = device_program(minors, has_kfd, kfd, !hide_kfd);
  static char license[] = "GPL";
  bpf_attr a{};
  a.prog_type = BPF_PROG_TYPE_CGROUP_DEVICE;
  a.insns = reinterpret_cast<uint64_t>(prog.data());
  a.insn_cnt = static_cast<uint32_t>(prog.size());
  a.license = reinterpret_cast<uint64_t>(license);
  int pfd = static_cast<int>(syscall(SYS_bpf, BPF_PROG_LOAD, &a, sizeof(a)));
  if (pfd < 0) {
    *err = std::string("bpf(PROG_LOAD cgroup_device): ") + std::strerror(errno);
    return false;
  }
  int cfd = open(cgroup_dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (cfd < 0) {
    *err = std::string("open cgroup ") + cgroup_dir + ": " + std::strerror(errno);
    close(pfd);
    return false;
  }
  bpf_attr at{};
  at.target_fd = static_cast<uint32_t>(cfd);
  at.attach_bpf_fd = static_cast<uint32_t>(pfd);
  at.attach_type = BPF_CGROUP_DEVICE;
  at.attach_flags = BPF_F_ALLOW_MULTI;
  bool ok = syscall(SYS_bpf, BPF_PROG_ATTACH, &at, sizeof(at)) == 0;
  if (!ok) *err = std::string("bpf(PROG_ATTACH cgroup_device): ") + std::strerror(errno);
  close(cfd);
  close(pfd);   // the attachment holds the program
  return ok;
}

}  // namespace amdkube_devguard
