// amdkube-bridge: the pod-network CNI plugin (CNI spec 0.3.1 / 0.4.0) behind rocshim's pod
// network namespaces — the kubenet equivalent (pkg/kubelet/network/kubenet: a `cbr0` bridge
// holding the node's pod-CIDR gateway, one veth pair per pod, host-local IPAM, hairpin mode,
// the MTU, lo up, a default route through the bridge) written directly against rtnetlink,
// with no `ip`/`brctl` binaries and no libnl.
//
//   {"cniVersion":"0.3.1","name":"podnet","type":"amdkube-bridge","bridge":"cbr0","mtu":1460,
//    "isGateway":true,"hairpinMode":true,
//    "ipam":{"type":"amdkube-cni","subnet":"10.244.1.0/24","dataDir":"..."}}
//
// ADD: delegate to the IPAM plugin (exec'd from CNI_PATH with the same config), ensure the
// bridge (up, gateway address when isGateway), create the veth pair with the peer born inside
// CNI_NETNS (IFLA_NET_NS_FD), enslave + hairpin + up the host end, then inside the namespace
// rename the peer to CNI_IFNAME, set MTU/address, bring it and lo up and add the default
// route; print the CNI result. DEL: IPAM DEL, then delete CNI_IFNAME inside the namespace
// (which removes the pair); both idempotent. CHECK: the interface carries an address.
//   amdkube-bridge --delete-bridge NAME   removes a bridge (node teardown / tests).
#include <arpa/inet.h>
#include <fcntl.h>
#include <linux/if_link.h>
#include <linux/netlink.h>
#include <linux/rtnetlink.h>
#include <linux/veth.h>
#include <net/if.h>
#include <sched.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#ifndef IFLA_BRPORT_MODE
#define IFLA_BRPORT_MODE 4
#endif

namespace {

// ---------------------------------------------------------------- minimal JSON field reader
std::string json_raw(const std::string& doc, const std::string& key) {
  std::string pat = "\"" + key + "\"";
  size_t p = doc.find(pat);
  if (p == std::string::npos) return "";
  p = doc.find(':', p + pat.size());
  if (p == std::string::npos) return "";
  p = doc.find_first_not_of(" \t\r\n", p + 1);
  if (p == std::string::npos) return "";
  if (doc[p] == '"') {
    std::string out;
    for (size_t i = p + 1; i < doc.size(); ++i) {
      if (doc[i] == '\\' && i + 1 < doc.size()) { out += doc[++i]; continue; }
      if (doc[i] == '"') return out;
      out += doc[i];
    }
    return "";
  }
  size_t e = doc.find_first_of(",}] \t\r\n", p);
  return doc.substr(p, e == std::string::npos ? std::string::npos : e - p);
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

std::string esc(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o;
}

int fail(int code, const std::string& msg, const std::string& version) {
  std::printf("{\"cniVersion\":\"%s\",\"code\":%d,\"msg\":\"%s\"}\n", version.c_str(), code, esc(msg).c_str());
  return 1;
}

// -------------------------------------------------------------------------- rtnetlink
struct Msg {
  std::vector<char> buf;
  explicit Msg(uint16_t type, uint16_t flags) : buf(NLMSG_SPACE(0), 0) {
    auto* h = hdr();
    h->nlmsg_len = NLMSG_LENGTH(0);
    h->nlmsg_type = type;
    h->nlmsg_flags = NLM_F_REQUEST | NLM_F_ACK | flags;
  }
  nlmsghdr* hdr() { return reinterpret_cast<nlmsghdr*>(buf.data()); }
  template <class T>
  T* put(const T& v) {  // fixed header (ifinfomsg / ifaddrmsg / rtmsg) right after nlmsghdr
    size_t off = NLMSG_ALIGN(hdr()->nlmsg_len);
    buf.resize(off + NLMSG_ALIGN(sizeof(T)), 0);
    std::memcpy(buf.data() + off, &v, sizeof(T));
    hdr()->nlmsg_len = off + sizeof(T);
    return reinterpret_cast<T*>(buf.data() + off);
  }
  size_t attr(uint16_t type, const void* data, size_t len) {
    size_t off = NLMSG_ALIGN(hdr()->nlmsg_len);
    buf.resize(off + RTA_SPACE(len), 0);
    auto* a = reinterpret_cast<rtattr*>(buf.data() + off);
    a->rta_type = type;
    a->rta_len = RTA_LENGTH(len);
    if (len) std::memcpy(RTA_DATA(a), data, len);
    hdr()->nlmsg_len = off + RTA_SPACE(len);
    return off;
  }
  size_t attr_str(uint16_t type, const std::string& s) { return attr(type, s.c_str(), s.size() + 1); }
  size_t attr_u32(uint16_t type, uint32_t v) { return attr(type, &v, 4); }
  size_t nest(uint16_t type) { return attr(type, nullptr, 0); }
  void end(size_t off) {
    auto* a = reinterpret_cast<rtattr*>(buf.data() + off);
    a->rta_len = hdr()->nlmsg_len - off;
  }
};

class Netlink {
 public:
  Netlink() { fd_ = socket(AF_NETLINK, SOCK_RAW | SOCK_CLOEXEC, NETLINK_ROUTE); }
  ~Netlink() { if (fd_ >= 0) close(fd_); }
  bool ok() const { return fd_ >= 0; }
  // returns 0 or -errno from the kernel's ack
  int call(Msg& m) {
    m.hdr()->nlmsg_seq = ++seq_;
    sockaddr_nl sa{};
    sa.nl_family = AF_NETLINK;
    if (sendto(fd_, m.buf.data(), m.hdr()->nlmsg_len, 0, reinterpret_cast<sockaddr*>(&sa), sizeof sa) < 0) return -errno;
    char rb[8192];
    for (;;) {
      ssize_t n = recv(fd_, rb, sizeof rb, 0);
      if (n < 0) return -errno;
      for (auto* h = reinterpret_cast<nlmsghdr*>(rb); NLMSG_OK(h, n); h = NLMSG_NEXT(h, n)) {
        if (h->nlmsg_seq != seq_) continue;
        if (h->nlmsg_type == NLMSG_ERROR) return reinterpret_cast<nlmsgerr*>(NLMSG_DATA(h))->error;
      }
    }
  }

 private:
  int fd_ = -1;
  uint32_t seq_ = 0;
};

ifinfomsg link_hdr(int index = 0, unsigned flags = 0, unsigned change = 0, unsigned char family = AF_UNSPEC) {
  ifinfomsg i{};
  i.ifi_family = family;
  i.ifi_index = index;
  i.ifi_flags = flags;
  i.ifi_change = change;
  return i;
}

int set_up(Netlink& nl, int index) {
  Msg m(RTM_NEWLINK, 0);
  m.put(link_hdr(index, IFF_UP, IFF_UP));
  return nl.call(m);
}

int set_mtu(Netlink& nl, int index, uint32_t mtu) {
  Msg m(RTM_NEWLINK, 0);
  m.put(link_hdr(index));
  m.attr_u32(IFLA_MTU, mtu);
  return nl.call(m);
}

int ensure_bridge(Netlink& nl, const std::string& name, uint32_t mtu) {
  if (if_nametoindex(name.c_str()) == 0) {
    Msg m(RTM_NEWLINK, NLM_F_CREATE | NLM_F_EXCL);
    m.put(link_hdr());
    m.attr_str(IFLA_IFNAME, name);
    if (mtu) m.attr_u32(IFLA_MTU, mtu);
    size_t li = m.nest(IFLA_LINKINFO);
    m.attr_str(IFLA_INFO_KIND, "bridge");
    m.end(li);
    int rc = nl.call(m);
    if (rc < 0 && rc != -EEXIST) return rc;
  }
  int idx = if_nametoindex(name.c_str());
  if (!idx) return -ENODEV;
  return set_up(nl, idx);
}

int add_addr(Netlink& nl, int index, uint32_t ip_be, int prefix) {
  Msg m(RTM_NEWADDR, NLM_F_CREATE | NLM_F_EXCL);
  ifaddrmsg a{};
  a.ifa_family = AF_INET;
  a.ifa_prefixlen = prefix;
  a.ifa_scope = RT_SCOPE_UNIVERSE;
  a.ifa_index = index;
  m.put(a);
  m.attr(IFA_LOCAL, &ip_be, 4);
  m.attr(IFA_ADDRESS, &ip_be, 4);
  int rc = nl.call(m);
  return rc == -EEXIST ? 0 : rc;
}

int create_veth(Netlink& nl, const std::string& host, const std::string& peer, int netns_fd, uint32_t mtu) {
  Msg m(RTM_NEWLINK, NLM_F_CREATE | NLM_F_EXCL);
  m.put(link_hdr());
  m.attr_str(IFLA_IFNAME, host);
  if (mtu) m.attr_u32(IFLA_MTU, mtu);
  size_t li = m.nest(IFLA_LINKINFO);
  m.attr_str(IFLA_INFO_KIND, "veth");
  size_t data = m.nest(IFLA_INFO_DATA);
  size_t p = m.nest(VETH_INFO_PEER);
  m.put(link_hdr());                        // the peer's ifinfomsg, then its attributes
  m.attr_str(IFLA_IFNAME, peer);
  if (mtu) m.attr_u32(IFLA_MTU, mtu);
  m.attr(IFLA_NET_NS_FD, &netns_fd, 4);
  m.end(p);
  m.end(data);
  m.end(li);
  return nl.call(m);
}

int set_master(Netlink& nl, int index, int master) {
  Msg m(RTM_NEWLINK, 0);
  m.put(link_hdr(index));
  m.attr_u32(IFLA_MASTER, master);
  return nl.call(m);
}

int set_hairpin(Netlink& nl, int index) {
  Msg m(RTM_SETLINK, 0);
  m.put(link_hdr(index, 0, 0, AF_BRIDGE));
  size_t pi = m.nest(IFLA_PROTINFO | NLA_F_NESTED);
  uint8_t on = 1;
  m.attr(IFLA_BRPORT_MODE, &on, 1);
  m.end(pi);
  return nl.call(m);
}

int rename_link(Netlink& nl, int index, const std::string& name) {
  Msg m(RTM_NEWLINK, 0);
  m.put(link_hdr(index));
  m.attr_str(IFLA_IFNAME, name);
  return nl.call(m);
}

int del_link(Netlink& nl, int index) {
  Msg m(RTM_DELLINK, 0);
  m.put(link_hdr(index));
  return nl.call(m);
}

int add_default_route(Netlink& nl, uint32_t gw_be, int oif) {
  Msg m(RTM_NEWROUTE, NLM_F_CREATE | NLM_F_EXCL);
  rtmsg r{};
  r.rtm_family = AF_INET;
  r.rtm_table = RT_TABLE_MAIN;
  r.rtm_protocol = RTPROT_BOOT;
  r.rtm_scope = RT_SCOPE_UNIVERSE;
  r.rtm_type = RTN_UNICAST;
  m.put(r);
  m.attr(RTA_GATEWAY, &gw_be, 4);
  m.attr_u32(RTA_OIF, oif);
  int rc = nl.call(m);
  return rc == -EEXIST ? 0 : rc;
}

std::string hex8(const std::string& s) {  // FNV-1a: stable per container, fits IFNAMSIZ
  uint32_t h = 2166136261u;
  for (unsigned char c : s) { h ^= c; h *= 16777619u; }
  char b[9];
  std::snprintf(b, sizeof b, "%08x", h);
  return b;
}

// run the IPAM plugin with our stdin and environment, capture stdout
int run_ipam(const std::string& type, const std::string& conf, std::string* out) {
  const char* path_env = std::getenv("CNI_PATH");
  std::string paths = path_env ? path_env : "", exe;
  size_t start = 0;
  while (start <= paths.size()) {
    size_t e = paths.find(':', start);
    std::string d = paths.substr(start, e == std::string::npos ? std::string::npos : e - start);
    if (!d.empty() && access((d + "/" + type).c_str(), X_OK) == 0) { exe = d + "/" + type; break; }
    if (e == std::string::npos) break;
    start = e + 1;
  }
  if (exe.empty()) { *out = "failed to find IPAM plugin " + type + " in CNI_PATH"; return -1; }
  int in[2], o[2];
  if (pipe(in) < 0 || pipe(o) < 0) return -1;
  pid_t pid = fork();
  if (pid == 0) {
    dup2(in[0], 0);
    dup2(o[1], 1);
    close(in[1]);
    close(o[0]);
    execl(exe.c_str(), exe.c_str(), static_cast<char*>(nullptr));
    _exit(127);
  }
  close(in[0]);
  close(o[1]);
  if (write(in[1], conf.data(), conf.size()) < 0) {}
  close(in[1]);
  char b[4096];
  ssize_t n;
  out->clear();
  while ((n = read(o[0], b, sizeof b)) > 0) out->append(b, n);
  close(o[0]);
  int st = 0;
  waitpid(pid, &st, 0);
  return WIFEXITED(st) ? WEXITSTATUS(st) : -1;
}

bool parse_cidr(const std::string& s, uint32_t* ip_be, int* prefix) {
  size_t sl = s.find('/');
  in_addr a{};
  if (sl == std::string::npos || inet_pton(AF_INET, s.substr(0, sl).c_str(), &a) != 1) return false;
  *ip_be = a.s_addr;
  *prefix = std::atoi(s.c_str() + sl + 1);
  return *prefix > 0 && *prefix <= 32;
}

int enter_netns(const std::string& path) {
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  int rc = setns(fd, CLONE_NEWNET) < 0 ? -errno : 0;
  close(fd);
  return rc;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc == 3 && std::string(argv[1]) == "--delete-bridge") {
    Netlink nl;
    int idx = if_nametoindex(argv[2]);
    if (!idx) return 0;
    int rc = del_link(nl, idx);
    if (rc < 0) std::fprintf(stderr, "delete %s: %s\n", argv[2], std::strerror(-rc));
    return rc < 0 ? 1 : 0;
  }
  const char* cmd_env = std::getenv("CNI_COMMAND");
  std::string cmd = cmd_env ? cmd_env : "";
  std::string conf((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
  std::string version = json_raw(conf, "cniVersion");
  if (version.empty()) version = "0.3.1";
  if (cmd == "VERSION") {
    std::printf("{\"cniVersion\":\"%s\",\"supportedVersions\":[\"0.3.0\",\"0.3.1\",\"0.4.0\"]}\n", version.c_str());
    return 0;
  }
  std::string netns = std::getenv("CNI_NETNS") ? std::getenv("CNI_NETNS") : "";
  std::string ifname = std::getenv("CNI_IFNAME") ? std::getenv("CNI_IFNAME") : "eth0";
  std::string cid = std::getenv("CNI_CONTAINERID") ? std::getenv("CNI_CONTAINERID") : "";
  if (cid.empty()) return fail(4, "CNI_CONTAINERID is required", version);
  std::string bridge = json_raw(conf, "bridge");
  if (bridge.empty()) bridge = "cbr0";
  uint32_t mtu = static_cast<uint32_t>(std::strtoul(json_raw(conf, "mtu").c_str(), nullptr, 10));
  bool gateway = json_raw(conf, "isGateway") == "true";
  bool hairpin = json_raw(conf, "hairpinMode") != "false";
  std::string ipam_type = json_raw(section(conf, "ipam"), "type");
  if (ipam_type.empty()) return fail(7, "missing ipam.type", version);

  if (cmd == "DEL") {
    std::string out;
    run_ipam(ipam_type, conf, &out);      // release the address whatever happens below
    if (!netns.empty() && enter_netns(netns) == 0) {
      Netlink nl;
      int idx = if_nametoindex(ifname.c_str());
      if (idx) del_link(nl, idx);          // deleting one end removes the pair
    }
    return 0;
  }
  if (netns.empty()) return fail(4, "CNI_NETNS is required", version);
  if (cmd == "CHECK") {
    if (enter_netns(netns) < 0) return fail(3, "cannot enter " + netns, version);
    if (!if_nametoindex(ifname.c_str())) return fail(3, "interface " + ifname + " missing", version);
    return 0;
  }
  if (cmd != "ADD") return fail(4, "unknown CNI_COMMAND " + cmd, version);

  std::string ipres;
  if (run_ipam(ipam_type, conf, &ipres) != 0) return fail(11, "IPAM " + ipam_type + " failed: " + ipres, version);
  uint32_t ip_be = 0, gw_be = 0;
  int prefix = 0;
  if (!parse_cidr(json_raw(ipres, "address"), &ip_be, &prefix)) return fail(11, "IPAM returned no address: " + ipres, version);
  std::string gws = json_raw(ipres, "gateway");
  in_addr ga{};
  if (!gws.empty() && inet_pton(AF_INET, gws.c_str(), &ga) == 1) gw_be = ga.s_addr;

  Netlink nl;
  if (!nl.ok()) return fail(11, std::string("netlink: ") + std::strerror(errno), version);
  int rc = ensure_bridge(nl, bridge, mtu);
  if (rc < 0) return fail(11, "bridge " + bridge + ": " + std::strerror(-rc), version);
  int br = if_nametoindex(bridge.c_str());
  if (gateway && gw_be) {
    rc = add_addr(nl, br, gw_be, prefix);
    if (rc < 0) return fail(11, "gateway address on " + bridge + ": " + std::strerror(-rc), version);
    int f = open("/proc/sys/net/ipv4/ip_forward", O_WRONLY | O_CLOEXEC);
    if (f >= 0) { if (write(f, "1", 1) < 0) {} close(f); }
  }
  std::string host_if = "veth" + hex8(cid + ifname), tmp_if = "tmp" + hex8(cid);
  int nsfd = open(netns.c_str(), O_RDONLY | O_CLOEXEC);
  if (nsfd < 0) return fail(11, "open " + netns + ": " + std::strerror(errno), version);
  if (int old = if_nametoindex(host_if.c_str())) del_link(nl, old);   // a stale pair from a failed ADD
  rc = create_veth(nl, host_if, tmp_if, nsfd, mtu);
  if (rc < 0) return fail(11, "veth " + host_if + ": " + std::strerror(-rc), version);
  int hidx = if_nametoindex(host_if.c_str());
  if ((rc = set_master(nl, hidx, br)) < 0) return fail(11, "enslave " + host_if + ": " + std::strerror(-rc), version);
  if (hairpin && (rc = set_hairpin(nl, hidx)) < 0) return fail(11, "hairpin " + host_if + ": " + std::strerror(-rc), version);
  if ((rc = set_up(nl, hidx)) < 0) return fail(11, "up " + host_if + ": " + std::strerror(-rc), version);

  if (setns(nsfd, CLONE_NEWNET) < 0) return fail(11, "setns " + netns + ": " + std::strerror(errno), version);
  close(nsfd);
  Netlink inner;                                // sockets belong to the netns they were made in
  int lo = if_nametoindex("lo");
  if (lo) set_up(inner, lo);
  int cidx = if_nametoindex(tmp_if.c_str());
  if (!cidx) return fail(11, "peer " + tmp_if + " missing in " + netns, version);
  if ((rc = rename_link(inner, cidx, ifname)) < 0) return fail(11, "rename to " + ifname + ": " + std::strerror(-rc), version);
  if (mtu) set_mtu(inner, cidx, mtu);
  if ((rc = add_addr(inner, cidx, ip_be, prefix)) < 0) return fail(11, "address: " + std::string(std::strerror(-rc)), version);
  if ((rc = set_up(inner, cidx)) < 0) return fail(11, "up " + ifname + ": " + std::strerror(-rc), version);
  if (gw_be && (rc = add_default_route(inner, gw_be, cidx)) < 0)
    return fail(11, "default route: " + std::string(std::strerror(-rc)), version);

  char ipb[INET_ADDRSTRLEN], gwb[INET_ADDRSTRLEN];
  inet_ntop(AF_INET, &ip_be, ipb, sizeof ipb);
  inet_ntop(AF_INET, &gw_be, gwb, sizeof gwb);
  std::printf("{\"cniVersion\":\"%s\",\"interfaces\":[{\"name\":\"%s\"},{\"name\":\"%s\"},{\"name\":\"%s\",\"sandbox\":\"%s\"}],"
              "\"ips\":[{\"version\":\"4\",\"address\":\"%s/%d\",\"gateway\":\"%s\",\"interface\":2}],"
              "\"routes\":[{\"dst\":\"0.0.0.0/0\",\"gw\":\"%s\"}],\"dns\":{}}\n",
              version.c_str(), esc(bridge).c_str(), host_if.c_str(), esc(ifname).c_str(), esc(netns).c_str(), ipb, prefix,
              gwb, gwb);
  return 0;
}
