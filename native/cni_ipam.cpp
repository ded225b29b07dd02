// amdkube-cni: a CNI (spec 0.3.1 / 0.4.0) plugin with host-local IPAM semantics.
//
// The reference delegates pod networking to CNI plugins exec'd by the kubelet's network
// plugin (pkg/kubelet/network/cni/cni.go: CNI_COMMAND / CNI_CONTAINERID / CNI_NETNS /
// CNI_IFNAME / CNI_ARGS / CNI_PATH in the environment, the network config on stdin, the
// result JSON on stdout, `{"code","msg"}` on failure) and ships `host-local` for address
// management (containernetworking/plugins ipam/host-local: one file per allocated IP named
// after the address and holding the container ID, `last_reserved_ip.<range>` for round
// robin, an flock'd lock file, the gateway and the network/broadcast addresses excluded).
//
// amdkube pods share the node's network namespace (the MI355X box runs unprivileged, so no
// veth / bridge set-up is possible), so this plugin is the IPAM: it gives every pod sandbox a
// unique, stable address from the node's pod CIDR, which the runtime reports as the pod IP
// that services and endpoints route to. It does not touch interfaces.
//
//   {"cniVersion":"0.3.1","name":"amdkube","type":"amdkube-cni",
//    "ipam":{"subnet":"10.244.1.0/24","rangeStart":"...","rangeEnd":"...","gateway":"...","dataDir":"..."}}
#include <arpa/inet.h>
#include <dirent.h>
#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <iterator>
#include <string>

namespace {

// ---- a minimal JSON field reader (the CNI config is small and flat enough) ----------------
std::string json_string(const std::string& doc, const std::string& key, size_t from = 0) {
  std::string pat = "\"" + key + "\"";
  size_t p = doc.find(pat, from);
  if (p == std::string::npos) return "";
  p = doc.find(':', p + pat.size());
  if (p == std::string::npos) return "";
  p = doc.find_first_not_of(" \t\r\n", p + 1);
  if (p == std::string::npos || doc[p] != '"') return "";
  std::string out;
  for (size_t i = p + 1; i < doc.size(); ++i) {
    if (doc[i] == '\\' && i + 1 < doc.size()) { out += doc[++i]; continue; }
    if (doc[i] == '"') return out;
    out += doc[i];
  }
  return "";
}

std::string section(const std::string& doc, const std::string& key) {
  size_t p = doc.find("\"" + key + "\"");
  if (p == std::string::npos) return "";
  p = doc.find('{', p);
  if (p == std::string::npos) return "";
  int depth = 0;
  for (size_t i = p; i < doc.size(); ++i) {
    if (doc[i] == '{') ++depth;
    else if (doc[i] == '}' && --depth == 0) return doc.substr(p, i - p + 1);
  }
  return "";
}

int fail(int code, const std::string& msg, const std::string& version) {
  std::printf("{\"cniVersion\":\"%s\",\"code\":%d,\"msg\":\"%s\"}\n", version.c_str(), code, msg.c_str());
  return 1;
}

bool parse_ip(const std::string& s, uint32_t* out) {
  in_addr a{};
  if (inet_pton(AF_INET, s.c_str(), &a) != 1) return false;
  *out = ntohl(a.s_addr);
  return true;
}

std::string ip_str(uint32_t v) {
  in_addr a{};
  a.s_addr = htonl(v);
  char b[INET_ADDRSTRLEN];
  inet_ntop(AF_INET, &a, b, sizeof b);
  return b;
}

std::string read_file(const std::string& p) {
  FILE* f = std::fopen(p.c_str(), "r");
  if (!f) return "";
  std::string s;
  char buf[256];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
  std::fclose(f);
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

bool write_file(const std::string& p, const std::string& s, bool exclusive) {
  int fd = open(p.c_str(), O_WRONLY | O_CREAT | (exclusive ? O_EXCL : O_TRUNC), 0644);
  if (fd < 0) return false;
  bool ok = write(fd, s.data(), s.size()) == static_cast<ssize_t>(s.size());
  close(fd);
  return ok;
}

void mkdirs(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i <= path.size(); ++i) {
    if (i == path.size() || path[i] == '/') {
      if (!cur.empty()) mkdir(cur.c_str(), 0755);
    }
    if (i < path.size()) cur += path[i];
  }
}

struct Range {
  uint32_t net = 0, mask = 0, start = 0, end = 0, gw = 0;
  int prefix = 0;
};

bool parse_range(const std::string& ipam, Range* r, std::string* err) {
  std::string subnet = json_string(ipam, "subnet");
  size_t slash = subnet.find('/');
  if (subnet.empty() || slash == std::string::npos) { *err = "ipam.subnet must be an IPv4 CIDR"; return false; }
  uint32_t base;
  if (!parse_ip(subnet.substr(0, slash), &base)) { *err = "invalid ipam.subnet address"; return false; }
  r->prefix = std::atoi(subnet.c_str() + slash + 1);
  if (r->prefix < 8 || r->prefix > 30) { *err = "ipam.subnet prefix must be in [8, 30]"; return false; }
  r->mask = r->prefix == 0 ? 0 : (0xffffffffu << (32 - r->prefix));
  r->net = base & r->mask;
  uint32_t bcast = r->net | ~r->mask;
  r->start = r->net + 1;
  r->end = bcast - 1;
  std::string s = json_string(ipam, "rangeStart"), e = json_string(ipam, "rangeEnd"), g = json_string(ipam, "gateway");
  uint32_t v;
  if (!s.empty() && parse_ip(s, &v) && (v & r->mask) == r->net) r->start = v;
  if (!e.empty() && parse_ip(e, &v) && (v & r->mask) == r->net) r->end = v;
  r->gw = r->net + 1;  // host-local default gateway: first address
  if (!g.empty() && parse_ip(g, &v)) r->gw = v;
  if (r->start > r->end) { *err = "empty allocation range"; return false; }
  return true;
}

}  // namespace

int main() {
  const char* cmd_env = std::getenv("CNI_COMMAND");
  std::string cmd = cmd_env ? cmd_env : "";
  std::string conf((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
  std::string version = json_string(conf, "cniVersion");
  if (version.empty()) version = "0.3.1";
  if (cmd == "VERSION") {
    std::printf("{\"cniVersion\":\"%s\",\"supportedVersions\":[\"0.3.0\",\"0.3.1\",\"0.4.0\"]}\n", version.c_str());
    return 0;
  }
  const char* cid_env = std::getenv("CNI_CONTAINERID");
  std::string cid = cid_env ? cid_env : "";
  if (cid.empty()) return fail(4, "CNI_CONTAINERID is required", version);
  std::string ipam = section(conf, "ipam");
  if (ipam.empty()) return fail(7, "missing ipam section", version);
  std::string name = json_string(conf, "name");
  if (name.empty()) name = "amdkube";
  std::string data_dir = json_string(ipam, "dataDir");
  if (data_dir.empty()) data_dir = "/var/lib/cni/networks";
  std::string dir = data_dir + "/" + name;
  mkdirs(dir);
  int lock = open((dir + "/lock").c_str(), O_RDWR | O_CREAT, 0644);
  if (lock < 0 || flock(lock, LOCK_EX) != 0) return fail(11, "cannot lock the IPAM store", version);

  auto owned_ip = [&](std::string* found) {
    DIR* d = opendir(dir.c_str());
    if (!d) return false;
    bool hit = false;
    while (dirent* e = readdir(d)) {
      uint32_t v;
      if (!parse_ip(e->d_name, &v)) continue;
      if (read_file(dir + "/" + e->d_name) == cid) { *found = e->d_name; hit = true; break; }
    }
    closedir(d);
    return hit;
  };

  if (cmd == "DEL") {
    std::string ip;
    while (owned_ip(&ip)) unlink((dir + "/" + ip).c_str());
    return 0;  // DEL is idempotent
  }
  Range r;
  std::string err;
  if (!parse_range(ipam, &r, &err)) return fail(7, err, version);
  std::string ip;
  if (cmd == "CHECK") {
    if (!owned_ip(&ip)) return fail(3, "no address allocated for " + cid, version);
    return 0;
  }
  if (cmd != "ADD") return fail(4, "unknown CNI_COMMAND " + cmd, version);
  if (!owned_ip(&ip)) {  // ADD is idempotent per container ID
    std::string last_file = dir + "/last_reserved_ip.0";
    uint32_t last = 0, cur;
    std::string l = read_file(last_file);
    if (l.empty() || !parse_ip(l, &last) || last < r.start || last > r.end) last = r.end;
    uint32_t n = r.end - r.start + 1;
    bool got = false;
    for (uint32_t i = 1; i <= n; ++i) {
      cur = r.start + (last - r.start + i) % n;
      if (cur == r.gw) continue;
      if (write_file(dir + "/" + ip_str(cur), cid, true)) { got = true; break; }
    }
    if (!got) return fail(11, "no IP addresses available in range " + ip_str(r.start) + "-" + ip_str(r.end), version);
    ip = ip_str(cur);
    write_file(last_file, ip, false);
  }
  std::printf("{\"cniVersion\":\"%s\",\"ips\":[{\"version\":\"4\",\"address\":\"%s/%d\",\"gateway\":\"%s\"}],"
              "\"routes\":[{\"dst\":\"0.0.0.0/0\"}],\"dns\":{}}\n",
              version.c_str(), ip.c_str(), r.prefix, ip_str(r.gw).c_str());
  close(lock);
  return 0;
}
