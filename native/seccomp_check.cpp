// seccomp-check: compile a profile and evaluate the resulting BPF program in user space.
//
//   seccomp-check PROFILE.json SYSCALL [ARG0 .. ARG5]   → prints the filter's return value
//   seccomp-check PROFILE.json --count                   → prints the program length
//
// It runs the same compiler as amdkube-nsexec through a classic-BPF interpreter covering the
// instructions the compiler emits, so tests can check rule order, the architecture guard
// and 64-bit argument comparisons exhaustively without executing the syscalls.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>

#include "seccomp_bpf.h"

static uint32_t run(const std::vector<sock_filter>& prog, const seccomp_data& d) {
  uint32_t A = 0;
  const auto* bytes = reinterpret_cast<const uint8_t*>(&d);
  for (size_t pc = 0; pc < prog.size(); ++pc) {
    const sock_filter& f = prog[pc];
    switch (f.code) {
      case BPF_LD | BPF_W | BPF_ABS:
        std::memcpy(&A, bytes + f.k, 4);
        break;
      case BPF_ALU | BPF_AND | BPF_K:
        A &= f.k;
        break;
      case BPF_JMP | BPF_JEQ | BPF_K:
        pc += (A == f.k) ? f.jt : f.jf;
        break;
      case BPF_JMP | BPF_JGT | BPF_K:
        pc += (A > f.k) ? f.jt : f.jf;
        break;
      case BPF_JMP | BPF_JGE | BPF_K:
        pc += (A >= f.k) ? f.jt : f.jf;
        break;
      case BPF_RET | BPF_K:
        return f.k;
      default:
        std::fprintf(stderr, "unexpected BPF opcode 0x%x at %zu\n", f.code, pc);
        std::exit(3);
    }
  }
  std::fprintf(stderr, "program fell off the end\n");
  std::exit(3);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: seccomp-check PROFILE SYSCALL [ARGS...] | PROFILE --count\n");
    return 2;
  }
  std::ifstream in(argv[1]);
  std::stringstream ss;
  ss << in.rdbuf();
  std::vector<sock_filter> prog;
  std::string err;
  if (!amdkube_seccomp::compile(ss.str(), &prog, &err)) {
    std::fprintf(stderr, "compile: %s\n", err.c_str());
    return 1;
  }
  if (std::string(argv[2]) == "--count") {
    std::printf("%zu\n", prog.size());
    return 0;
  }
  seccomp_data d{};
  d.arch = AUDIT_ARCH_X86_64;
  int nr = amdkube_seccomp::syscall_number(argv[2]);
  d.nr = nr >= 0 ? nr : std::atoi(argv[2]);
  if (argc > 3 && std::string(argv[3]) == "--arch") {   // evaluate a foreign-ABI entry
    d.arch = static_cast<uint32_t>(std::strtoul(argv[4], nullptr, 0));
    argv += 2;
    argc -= 2;
  }
  for (int i = 3; i < argc && i - 3 < 6; ++i) d.args[i - 3] = std::strtoull(argv[i], nullptr, 0);
  std::printf("0x%08" PRIx32 "\n", run(prog, d));
  return 0;
}
