// codescan.cpp — what a compiled segmented-walk code object does with scratch.
//
// The segmented walk's live-value budget is checked against the compiler
// (jit.cpp build_seg): a budget is acceptable only if the kernel's walk loop
// — the loop that runs 2^m / 2^(b+1) times per wave-chunk — touches no scratch.
// A spill in the chunk start costs a few accesses per 2^m Gray steps; one in
// the walk loop runs on every shared step.  The metadata's VGPR spill count
// cannot tell the two apart, so the kernel is disassembled (amd_comgr, the
// disassembler hiprtc itself ships with) and its control-flow graph analysed:
// basic blocks, dominators (Cooper-Harvey-Kennedy), natural loops of the back
// edges.  The walk loop is the loop with the most fp64 VALU instructions that
// holds no inner loop carrying half of them or more (the chunk loop around
// it does); its scratch_* / buffer_* instructions are counted.
#include <amd_comgr/amd_comgr.h>
#include <elf.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <string_view>
#include <vector>

#include "engine.hpp"

namespace sup {

namespace {

struct Inst {
  uint64_t addr = 0, size = 0;
  std::string text;        // mnemonic and operands
  int64_t target = -1;     // branch target (absolute address), -1 if none
};

struct DisCtx {
  const char* bytes = nullptr;  // section contents
  uint64_t base = 0, len = 0;   // virtual address range of the section
  std::string text;
  int64_t target = -1;
};

uint64_t read_cb(uint64_t from, char* to, uint64_t size, void* user) {
  DisCtx& c = *(DisCtx*)user;
  if (from < c.base || from >= c.base + c.len) return 0;
  const uint64_t n = std::min(size, c.base + c.len - from);
  std::memcpy(to, c.bytes + (from - c.base), n);
  return n;
}
void print_cb(const char* inst, void* user) { ((DisCtx*)user)->text = inst; }
void annot_cb(uint64_t addr, void* user) { ((DisCtx*)user)->target = (int64_t)addr; }

// Unsigned msgpack value after the map key `key` in the metadata note (fixstr
// key; fixint / uint8-32 value); -1 if absent.
long meta_value(const std::vector<char>& co, const std::string& key) {
  if (key.size() >= 32) return -1;
  std::string pat(1, (char)(0xa0 | key.size()));
  pat += key;
  const std::string_view sv(co.data(), co.size());
  const size_t at = sv.find(pat);
  if (at == std::string_view::npos || at + pat.size() >= co.size()) return -1;
  const unsigned char* v = (const unsigned char*)co.data() + at + pat.size();
  const size_t left = co.size() - at - pat.size();
  if (v[0] < 0x80) return v[0];
  if (v[0] == 0xcc && left >= 2) return v[1];
  if (v[0] == 0xcd && left >= 3) return (v[1] << 8) | v[2];
  if (v[0] == 0xce && left >= 5) return ((long)v[1] << 24) | (v[2] << 16) | (v[3] << 8) | v[4];
  return -1;
}

// Section bytes and virtual range of function `name` in an ELF64 code object.
bool find_function(const std::vector<char>& co, const char* name, const char** bytes, uint64_t* addr,
                   uint64_t* size, uint64_t* sec_addr, uint64_t* sec_len) {
  if (co.size() < sizeof(Elf64_Ehdr)) return false;
  Elf64_Ehdr eh;
  std::memcpy(&eh, co.data(), sizeof eh);
  if (std::memcmp(eh.e_ident, ELFMAG, SELFMAG) != 0 || eh.e_ident[EI_CLASS] != ELFCLASS64) return false;
  if (eh.e_shoff == 0 || eh.e_shentsize != sizeof(Elf64_Shdr) ||
      eh.e_shoff + (uint64_t)eh.e_shnum * sizeof(Elf64_Shdr) > co.size())
    return false;
  std::vector<Elf64_Shdr> sh(eh.e_shnum);
  std::memcpy(sh.data(), co.data() + eh.e_shoff, sh.size() * sizeof(Elf64_Shdr));
  for (const Elf64_Shdr& s : sh) {
    if (s.sh_type != SHT_SYMTAB || s.sh_link >= sh.size() || s.sh_entsize != sizeof(Elf64_Sym)) continue;
    const Elf64_Shdr& str = sh[s.sh_link];
    if (s.sh_offset + s.sh_size > co.size() || str.sh_offset + str.sh_size > co.size()) return false;
    for (uint64_t i = 0; i < s.sh_size / sizeof(Elf64_Sym); ++i) {
      Elf64_Sym sym;
      std::memcpy(&sym, co.data() + s.sh_offset + i * sizeof(Elf64_Sym), sizeof sym);
      if (ELF64_ST_TYPE(sym.st_info) != STT_FUNC || sym.st_name >= str.sh_size || sym.st_shndx >= sh.size())
        continue;
      const char* nm = co.data() + str.sh_offset + sym.st_name;
      if (std::strncmp(nm, name, str.sh_size - sym.st_name) != 0) continue;
      const Elf64_Shdr& text = sh[sym.st_shndx];
      if (text.sh_offset + text.sh_size > co.size() || sym.st_value < text.sh_addr ||
          sym.st_value + sym.st_size > text.sh_addr + text.sh_size)
        return false;
      *bytes = co.data() + text.sh_offset;
      *sec_addr = text.sh_addr;
      *sec_len = text.sh_size;
      *addr = sym.st_value;
      *size = sym.st_size;
      return true;
    }
  }
  return false;
}

bool starts(const std::string& s, const char* p) { return s.compare(0, std::strlen(p), p) == 0; }

bool is_f64_valu(const std::string& t) {
  return starts(t, "v_add_f64") || starts(t, "v_mul_f64") || starts(t, "v_fma_f64") || starts(t, "v_fmac_f64");
}
bool is_scratch(const std::string& t) { return starts(t, "scratch_") || starts(t, "buffer_"); }
// SGPR spill reloads: the allocator parks SGPRs in VGPR lanes (v_writelane) and
// reads them back with v_readlane, a VALU instruction in the fp64 stream
bool is_readlane(const std::string& t) { return starts(t, "v_readlane"); }

}  // namespace

int scan_code_object(const std::vector<char>& co, const char* kernel, CodeScan* out) {
  CodeScan r;
  r.vgprs = (int)meta_value(co, ".vgpr_count");
  r.vgpr_spills = (int)meta_value(co, ".vgpr_spill_count");
  r.scratch_bytes = (int)meta_value(co, ".private_segment_fixed_size");
  if (r.vgprs < 0 || r.vgpr_spills < 0 || r.scratch_bytes < 0) {
    set_error("code object: no register / scratch counts in its metadata");
    return SUP_EHIP;
  }
  const char* bytes = nullptr;
  uint64_t fa = 0, fs = 0, sa = 0, sl = 0;
  if (!find_function(co, kernel, &bytes, &fa, &fs, &sa, &sl) || fs == 0) {
    set_error(std::string("code object: kernel symbol ") + kernel + " not found");
    return SUP_EHIP;
  }
  // ---- disassemble
  DisCtx ctx;
  ctx.bytes = bytes, ctx.base = sa, ctx.len = sl;
  amd_comgr_disassembly_info_t dis;
  if (amd_comgr_create_disassembly_info("amdgcn-amd-amdhsa--gfx950", read_cb, print_cb, annot_cb, &dis) !=
      AMD_COMGR_STATUS_SUCCESS) {
    set_error("amd_comgr_create_disassembly_info failed");
    return SUP_EHIP;
  }
  std::vector<Inst> ins;
  int rc = SUP_OK;
  for (uint64_t a = fa; a < fa + fs;) {
    ctx.text.clear();
    ctx.target = -1;
    uint64_t sz = 0;
    if (amd_comgr_disassemble_instruction(dis, a, &ctx, &sz) != AMD_COMGR_STATUS_SUCCESS || sz == 0) {
      set_error("code object: disassembly failed");
      rc = SUP_EHIP;
      break;
    }
    Inst in;
    in.addr = a, in.size = sz;
    size_t p = ctx.text.find_first_not_of(" \t");
    in.text = p == std::string::npos ? std::string() : ctx.text.substr(p);
    const bool branch = starts(in.text, "s_branch") || starts(in.text, "s_cbranch");
    in.target = branch ? ctx.target : -1;
    ins.push_back(std::move(in));
    a += sz;
  }
  amd_comgr_destroy_disassembly_info(dis);
  if (rc) return rc;
  for (const Inst& in : ins) r.scratch_insts += is_scratch(in.text);
  r.insts = (int)ins.size();

  // ---- basic blocks
  std::map<uint64_t, int> at;  // address -> instruction index
  for (size_t i = 0; i < ins.size(); ++i) at[ins[i].addr] = (int)i;
  std::vector<char> leader(ins.size() + 1, 0);
  leader[0] = 1;
  for (size_t i = 0; i < ins.size(); ++i) {
    const Inst& in = ins[i];
    const bool ends = in.target >= 0 || starts(in.text, "s_endpgm") || starts(in.text, "s_setpc");
    if (ends) leader[i + 1] = 1;
    if (in.target >= 0) {
      auto it = at.find((uint64_t)in.target);
      if (it == at.end()) {
        set_error("code object: branch target outside the kernel");
        return SUP_EHIP;
      }
      leader[it->second] = 1;
    }
  }
  std::vector<int> bstart, block_of(ins.size());
  for (size_t i = 0; i < ins.size(); ++i) {
    if (leader[i]) bstart.push_back((int)i);
    block_of[i] = (int)bstart.size() - 1;
  }
  const int B = (int)bstart.size();
  std::vector<std::vector<int>> succ(B), pred(B);
  std::vector<int> bf64(B, 0), bscr(B, 0), blen(B, 0), brl(B, 0);
  for (int b = 0; b < B; ++b) {
    const int lo = bstart[b], hi = b + 1 < B ? bstart[b + 1] : (int)ins.size();
    for (int i = lo; i < hi; ++i)
      bf64[b] += is_f64_valu(ins[i].text), bscr[b] += is_scratch(ins[i].text), brl[b] += is_readlane(ins[i].text);
    blen[b] = hi - lo;
    const Inst& last = ins[hi - 1];
    auto add = [&](int to) {
      if (to >= 0 && to < B) succ[b].push_back(to), pred[to].push_back(b);
    };
    if (last.target >= 0) add(block_of[at[(uint64_t)last.target]]);
    const bool uncond = starts(last.text, "s_branch") || starts(last.text, "s_endpgm") || starts(last.text, "s_setpc");
    if (!uncond && hi < (int)ins.size()) add(b + 1);
  }
  // ---- dominators (reverse post-order, iterative)
  std::vector<int> order, rpo_num(B, -1);
  {
    std::vector<char> seen(B, 0);
    std::vector<std::pair<int, size_t>> st{{0, 0}};
    seen[0] = 1;
    while (!st.empty()) {
      auto& [v, k] = st.back();
      if (k < succ[v].size()) {
        const int w = succ[v][k++];
        if (!seen[w]) seen[w] = 1, st.push_back({w, 0});
      } else {
        order.push_back(v);
        st.pop_back();
      }
    }
    std::reverse(order.begin(), order.end());
    for (size_t i = 0; i < order.size(); ++i) rpo_num[order[i]] = (int)i;
  }
  std::vector<int> idom(B, -1);
  idom[0] = 0;
  auto intersect = [&](int a, int b) {
    while (a != b) {
      while (rpo_num[a] > rpo_num[b]) a = idom[a];
      while (rpo_num[b] > rpo_num[a]) b = idom[b];
    }
    return a;
  };
  for (bool changed = true; changed;) {
    changed = false;
    for (int v : order) {
      if (v == 0) continue;
      int nd = -1;
      for (int p : pred[v])
        if (rpo_num[p] >= 0 && idom[p] >= 0) nd = nd < 0 ? p : intersect(p, nd);
      if (nd >= 0 && idom[v] != nd) idom[v] = nd, changed = true;
    }
  }
  auto dominates = [&](int h, int v) {
    if (rpo_num[v] < 0) return false;
    for (;;) {
      if (v == h) return true;
      if (v == 0) return false;
      v = idom[v];
    }
  };
  // ---- natural loops, merged by header
  std::map<int, std::vector<char>> loops;
  for (int u = 0; u < B; ++u)
    for (int h : succ[u]) {
      if (!dominates(h, u)) continue;
      std::vector<char>& body = loops[h];
      if (body.empty()) body.assign(B, 0);
      body[h] = 1;
      std::vector<int> work;
      if (!body[u]) body[u] = 1, work.push_back(u);
      while (!work.empty()) {
        const int v = work.back();
        work.pop_back();
        for (int p : pred[v])
          if (!body[p]) body[p] = 1, work.push_back(p);
      }
    }
  r.loops = (int)loops.size();
  // ---- the walk loop: most fp64 work, no inner loop holding half of it
  std::map<int, int> f64;
  for (auto& [h, body] : loops) {
    int s = 0;
    for (int b = 0; b < B; ++b) s += body[b] ? bf64[b] : 0;
    f64[h] = s;
  }
  int walk = -1;
  for (auto& [h, body] : loops) {
    bool outer = false;
    for (auto& [h2, body2] : loops)
      if (h2 != h && body[h2] && 2 * f64[h2] >= f64[h]) outer = true;
    if (!outer && (walk < 0 || f64[h] > f64[walk])) walk = h;
  }
  if (walk >= 0) {
    const std::vector<char>& body = loops[walk];
    r.loop_f64 = f64[walk];
    r.loop_scratch = 0;
    r.loop_insts = 0;
    r.loop_readlane = 0;
    for (int b = 0; b < B; ++b)
      if (body[b]) r.loop_scratch += bscr[b], r.loop_insts += blen[b], r.loop_readlane += brl[b];
  }
  *out = r;
  return SUP_OK;
}

}  // namespace sup
