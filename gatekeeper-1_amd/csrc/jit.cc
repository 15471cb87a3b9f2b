// Template JIT (see jit.h).
#include "jit.h"

#include <hip/hiprtc.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <set>
#include <sstream>
#include <sys/stat.h>
#include <unistd.h>

// device runtime sources, embedded at build time (Makefile: build/rtsrc.cc)
extern const char gk_rt_common_h[];
extern const char gk_rt_devrt_h[];

namespace gk {
namespace {

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h;
}

const char* kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-w"};
constexpr int kNOpts = 4;

std::string hex16(uint64_t v) {
  char b[17];
  snprintf(b, sizeof b, "%016llx", (unsigned long long)v);
  return b;
}

// Body of the predicate function: one statement per bytecode instruction.
// Unlike the VM, the generated code does not test L.fail after every helper
// call (a scratch load per call): the first failure recorded in the lane wins
// either way, helpers return well-formed values (undefined) once it is set,
// and a failed lane's staged tuples are discarded by flush_wave — so running
// on to the end yields the same lane outcome at no cost to passing lanes.
std::string body(const Program& p, const CodeBank& bank) {
  const uint32_t b0 = p.code_off, b1 = p.code_off + p.code_len;
  std::set<uint32_t> labels, memo;
  for (uint32_t pc = b0; pc < b1; ++pc) {
    const Ins& in = bank.code[pc];
    switch (in.op) {
      case OP_JMP: case OP_JUNDEF: case OP_JFALSE: case OP_JTRUE: case OP_ITER_NEXT: case OP_MEMO_GET:
        labels.insert(in.x);
        break;
      default: break;
    }
    if (in.op == OP_MEMO_GET || in.op == OP_MEMO_PUT) memo.insert(in.y);
  }
  std::ostringstream o;
  auto R = [](uint32_t r) { return "r" + std::to_string(r); };
  // no initializers: the compiler writes every register before reading it (the
  // VM kernel relies on the same), and zero-initialising would make all of them
  // live from entry — register pressure, hence occupancy
  o << "  uint64_t ";
  for (uint32_t r = 0; r < p.nregs; ++r) o << (r ? ", " : "") << R(r);
  if (!p.nregs) o << "unused_";
  o << ";\n";
  // memo slots are locals too: (key0, key1, value, valid)
  for (uint32_t m : memo)
    o << "  uint64_t mk0_" << m << ", mk1_" << m << ", mv_" << m << "; bool mok_" << m << " = false;\n";
  const char* UND = "0x0000000000000000ull";
  char kb[40];
  auto lit = [&](uint64_t v) { snprintf(kb, sizeof kb, "0x%016llxull", (unsigned long long)v); return std::string(kb); };
  for (uint32_t pc = b0; pc < b1; ++pc) {
    const Ins& in = bank.code[pc];
    if (labels.count(pc)) o << "L" << pc << ":;\n";
    std::string a = R(in.a), b = R(in.b), c = R(in.c), x = "L" + std::to_string(in.x);
    std::string y = std::to_string(in.y) + "u";
    o << "  ";
    switch (in.op) {
      case OP_END: o << "return;"; break;
      case OP_JMP: o << "goto " << x << ";"; break;
      case OP_JUNDEF: o << "if (vtag(" << a << ") == V_UNDEF) goto " << x << ";"; break;
      case OP_JFALSE: o << "if (" << a << " == " << lit(((uint64_t)V_BOOL << 60) | 0) << ") goto " << x << ";"; break;
      case OP_JTRUE: o << "if (" << a << " == " << lit(((uint64_t)V_BOOL << 60) | 1) << ") goto " << x << ";"; break;
      case OP_LOADK: o << a << " = " << lit(bank.consts[in.x]) << ";"; break;
      case OP_LOADREV: o << a << " = review;"; break;
      case OP_LOADPARAM: o << a << " = params;"; break;
      case OP_MOV: o << a << " = " << b << ";"; break;
      case OP_GET: o << a << " = vget(L, " << b << ", " << c << ");"; break;
      case OP_GETK: o << a << " = vget(L, " << b << ", " << lit(bank.consts[in.x]) << ");"; break;
      case OP_ITER_INIT: o << "op_iter_init(L, " << a << ", " << R(in.a + 1) << ", " << b << ", " << y << ");"; break;
      case OP_ITER_NEXT:
        o << "{ uint64_t k_ = " << UND << ", v_ = " << UND << "; if (!op_iter_next(L, " << a << ", " << R(in.a + 1)
          << ", " << y << ", k_, v_)) goto " << x << ";";
        if (in.b != 0xffff) o << " " << b << " = k_;";
        if (in.c != 0xffff) o << " " << c << " = v_;";
        o << " }";
        break;
      case OP_CMP: o << "if (!op_cmp(L, " << y << ", " << b << ", " << c << ", " << a << ")) return;"; break;
      case OP_ARITH: o << a << " = arith(L, " << y << ", " << b << ", " << c << ");"; break;
      case OP_LIST_NEW: o << a << " = list_new(L, " << y << ", 4);"; break;
      case OP_LIST_ADD: o << "if (!op_list_add(L, " << a << ", " << b << ", " << y << ")) return;"; break;
      case OP_OBJ_PUT: o << "if (!op_obj_put(L, " << a << ", " << b << ", " << c << ", " << y << ")) return;"; break;
      case OP_YIELD: o << "if (!op_yield(L, " << a << ", " << b << ", " << y << ")) return;"; break;
      case OP_CALL: {
        uint32_t n = in.c ? in.c : 1;
        o << "{ uint64_t av_[" << n << "] = {";
        for (uint32_t i = 0; i < in.c; ++i) o << (i ? ", " : "") << R(in.b + i);
        if (!in.c) o << "0";
        o << "}; " << a << " = call_builtin(L, " << y << ", av_); }";
        break;
      }
      case OP_SPRINTF: o << a << " = do_sprintf(L, " << in.x << "u, " << b << ");"; break;
      case OP_LEN_EQ: o << a << " = op_len_eq(L, " << b << ", " << y << ");"; break;
      case OP_EMIT:
        o << "if (!op_emit(L, " << a << ", " << (in.b == 0xffff ? std::string(UND) : b) << ", " << in.c << "u, " << y
          << ")) return;";
        break;
      case OP_MEMO_GET: {
        std::string m = std::to_string(in.y), k1 = in.c == 0xffff ? std::string("0ull") : c;
        o << "if (mok_" << m << " && mk0_" << m << " == " << b << " && mk1_" << m << " == " << k1 << ") { " << a
          << " = mv_" << m << "; goto " << x << "; }";
        break;
      }
      case OP_MEMO_PUT: {
        std::string m = std::to_string(in.y), k1 = in.c == 0xffff ? std::string("0ull") : c;
        o << "if (memo_stable(" << b << ") && memo_stable(" << k1 << ") && memo_stable(" << a << ")) { mk0_" << m
          << " = " << b << "; mk1_" << m << " = " << k1 << "; mv_" << m << " = " << a << "; mok_" << m << " = true; }";
        break;
      }
      case OP_TABLE: o << a << " = op_table(L, gk_args.K + " << in.x << "u, " << b << ");"; break;
      case OP_FAIL_FALLBACK: o << "lane_fallback(L, " << y << "); return;"; break;
      default: o << "lane_fallback(L, FB_UNSUPPORTED); return;"; break;
    }
    o << "\n";
  }
  o << "  lane_fallback(L, FB_UNSUPPORTED);\n";
  return o.str();
}

std::mutex g_mu;
std::map<std::string, std::string> g_cache;  // source -> code object

std::string cache_dir() {
  const char* d = getenv("GKGPU_JIT_CACHE");
  if (d && !strcmp(d, "0")) return "";
  if (d && *d) return d;
  const char* h = getenv("HOME");
  if (!h || !*h) return "";
  return std::string(h) + "/.cache/gkgpu-jit";
}

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return !out.empty();
}

void write_file_atomic(const std::string& dir, const std::string& name, const std::string& data) {
  std::string cur;
  for (size_t i = 1; i <= dir.size(); ++i)
    if (i == dir.size() || dir[i] == '/') { cur = dir.substr(0, i); mkdir(cur.c_str(), 0755); }
  std::string tmp = dir + "/." + name + "." + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    if (!f) return;
    f.write(data.data(), (std::streamsize)data.size());
    if (!f) { unlink(tmp.c_str()); return; }
  }
  if (rename(tmp.c_str(), (dir + "/" + name).c_str()) != 0) unlink(tmp.c_str());
}

}  // namespace

// Minimum waves per SIMD the template kernels are compiled for (caps VGPRs at
// 512/n; the compiler spills beyond).  Default 2: measured on config 2 (1M Pods,
// MI355X), K8sContainerLimits 65 ms at the compiler's own choice (1 wave, 248
// VGPRs), 41 ms at 2 (256 VGPRs, 8 spills), 69 ms at 4 (128 VGPRs, heavy
// spills).  GKGPU_JIT_WPE overrides (0 = compiler's choice).
static std::string wpe_suffix() {
  const char* w = getenv("GKGPU_JIT_WPE");
  int n = w ? atoi(w) : 2;
  return n > 0 ? ", " + std::to_string(n) : std::string();
}

std::string jit_name(const Program& p, const CodeBank& bank) {
  return "gk_t_" + hex16(fnv1a(body(p, bank) + wpe_suffix()));
}

std::string jit_source(const Program& p, const CodeBank& bank, const std::string& name) {
  std::ostringstream o;
  o << "// generated by jit.cc from template bytecode (" << p.code_len << " instructions)\n"
    << "#include \"devrt.h\"\n"
    << "namespace gk {\n"
    << "__device__ void " << name << "_pred(Lane& L, uint64_t review, uint64_t params) {\n"
    << body(p, bank) << "}\n"
    << "}  // namespace gk\n"
    << "extern \"C\" __global__ void __launch_bounds__(256" << wpe_suffix() << ") " << name << "() {\n"
    << "  gk::audit_body([&](gk::Lane& L, uint64_t review, uint64_t params, uint32_t, uint32_t, uint32_t) {\n"
    << "    gk::" << name << "_pred(L, review, params);\n"
    << "  });\n"
    << "}\n";
  return o.str();
}

bool jit_compile(const std::string& src, std::string& code, std::string& log) {
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_cache.find(src);
    if (it != g_cache.end()) { code = it->second; return true; }
  }
  int ver_major = 0, ver_minor = 0;
  hiprtcVersion(&ver_major, &ver_minor);
  std::string key = hex16(fnv1a(src, fnv1a(std::string(gk_rt_common_h) + gk_rt_devrt_h +
                                           std::to_string(ver_major) + "." + std::to_string(ver_minor))));
  std::string dir = cache_dir();
  std::string fname = key + ".co";
  if (!dir.empty() && read_file(dir + "/" + fname, code)) {
    std::lock_guard<std::mutex> g(g_mu);
    g_cache[src] = code;
    return true;
  }
  if (const char* dd = getenv("GKGPU_JIT_DUMP")) {  // diagnostics: keep the generated source
    if (*dd) write_file_atomic(dd, key + ".hip", src);
  }
  hiprtcProgram prog;
  const char* hs[] = {gk_rt_common_h, gk_rt_devrt_h};
  const char* hn[] = {"common.h", "devrt.h"};
  if (hiprtcCreateProgram(&prog, src.c_str(), "gk_template.hip", 2, hs, hn) != HIPRTC_SUCCESS) {
    log = "hiprtcCreateProgram failed";
    return false;
  }
  hiprtcResult r = hiprtcCompileProgram(prog, kNOpts, kOpts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  log.assign(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &log[0]);
  bool ok = r == HIPRTC_SUCCESS;
  if (ok) {
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.assign(cs, '\0');
    ok = cs > 0 && hiprtcGetCode(prog, &code[0]) == HIPRTC_SUCCESS;
  }
  hiprtcDestroyProgram(&prog);
  if (!ok) return false;
  {
    std::lock_guard<std::mutex> g(g_mu);
    g_cache[src] = code;
  }
  if (!dir.empty()) write_file_atomic(dir, fname, code);
  return true;
}

}  // namespace gk
