// qpb_hazard.cpp -- manual wait states for the DPP inline asm of the row / wave
// kernels (gfx950).
//
// The kernels issue v_fmac_f64_dpp from inline asm (the compiler does not fold a
// 64-bit DPP move into an FMA).  The compiler's hazard recognizer cannot look
// into inline asm, so the wait states a DPP instruction needs are ours to place:
//   * 2 after a VALU write of ANY VGPR the DPP instruction reads -- the permuted
//     source, the other source and the tied accumulator (the rule LLVM's
//     GCNHazardRecognizer::checkDPPHazards applies to its own DPP code);
//   * 5 after a VALU write of EXEC (v_cmpx);
//   * kMfmaWs after an MFMA writes such a VGPR (its result lands late; the value
//     is generous for every gfx950 MFMA shape, none of ours feeds DPP directly).
// The audit over the whole code object checks two more gfx950 hazard classes, on every
// instruction (compiler-generated code included -- a finding there would be a backend
// gap; none exists in any kernel of this repository):
//   * trans forwarding: a VALU instruction reading a VGPR written by a transcendental
//     (v_rcp / v_rsq / v_sqrt / v_exp / v_log / v_sin / v_cos) needs 1 wait state --
//     an inline-asm consumer of a v_rcp_f64 result gets none from the compiler;
//   * a VMEM instruction reading an SGPR (its saddr / soffset) that a VALU wrote
//     (v_readlane, v_readfirstlane, v_cmp into an SGPR pair, carry-outs) needs 5 -- a
//     stale base would be a wrong (possibly illegal) address.
// asm_fixup pads the inline-asm DPP instructions for the trans rule as well.
// Two users of one scan:
//   * asm_fixup: compiling a kernel with DPP asm goes through assembly (clang -S);
//     every DPP instruction inside an inline-asm region gets exactly the s_nop it
//     needs on every path into it (branches and loop back-edges included), then
//     the text is assembled and linked;
//   * audit: the same check over the disassembled code object (llvm-objdump),
//     run on every code object before it is cached.
#include "qpb_hazard.hpp"

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <sstream>
#include <vector>

namespace qpb {
namespace {

constexpr int kDppVgprWs = 2, kDppExecWs = 5, kMfmaWs = 19, kTransWs = 1, kSgprVmemWs = 5, kMaxWs = kMfmaWs;
enum Rules { R_DPP = 1, R_TRANS = 2, R_SGPR_VMEM = 4 };

struct Insn {
    std::string mn;
    std::vector<std::pair<int, int>> vregs;   // every v register operand, [lo, hi], in operand order
    std::vector<std::pair<int, int>> vreads;  // the VGPRs it reads (operand 0 only for mac / fmac / DPP)
    std::vector<std::pair<int, int>> sregs;   // every s register operand (vcc as s1000:1001)
    std::vector<std::pair<int, int>> sdefs;   // SGPRs a VALU instruction writes
    bool valu = false, trans = false, vmem = false;
    bool vdef0 = false;                       // first operand is a VGPR the instruction writes (VALU)
    bool mfma = false;
    bool exec_valu_def = false;               // v_cmpx*: VALU write of EXEC
    bool dpp = false;                         // a DPP instruction this pass is responsible for
    bool uncond = false;                      // no fall-through
    int ws = 1;                               // wait states the instruction itself provides
    std::string target;                       // branch target (label or address)
    size_t line = 0;                          // source line (asm_fixup)
};

bool parse_vreg(const std::string &t, std::pair<int, int> &r) {
    size_t i = 0;
    while (i < t.size() && (t[i] == ' ' || t[i] == '\t' || t[i] == '-' || t[i] == '|')) i++;
    if (i + 1 >= t.size() || t[i] != 'v') return false;
    if (t[i + 1] == '[') {
        int a = 0, b = 0;
        if (sscanf(t.c_str() + i + 2, "%d:%d]", &a, &b) != 2) return false;
        r = {a, b};
        return true;
    }
    if (!isdigit((unsigned char)t[i + 1])) return false;
    const int a = atoi(t.c_str() + i + 1);
    r = {a, a};
    return true;
}

bool parse_sreg(const std::string &t, std::pair<int, int> &r) {
    size_t i = 0;
    while (i < t.size() && (t[i] == ' ' || t[i] == '\t' || t[i] == '-' || t[i] == '|')) i++;
    if (t.compare(i, 3, "vcc") == 0) { r = {1000, 1001}; return true; }
    if (i + 1 >= t.size() || t[i] != 's') return false;
    if (t[i + 1] == '[') {
        int a = 0, b = 0;
        if (sscanf(t.c_str() + i + 2, "%d:%d]", &a, &b) != 2) return false;
        r = {a, b};
        return true;
    }
    if (!isdigit((unsigned char)t[i + 1])) return false;
    const int a = atoi(t.c_str() + i + 1);
    r = {a, a};
    return true;
}

// one instruction's text "mnemonic op, op, op modifiers..."
Insn parse_insn(const std::string &text) {
    Insn a;
    std::istringstream ts(text);
    ts >> a.mn;
    std::string rest;
    std::getline(ts, rest);
    std::vector<std::string> ops;
    {
        std::string cur;
        for (char ch : rest) {
            if (ch == ',') { ops.push_back(cur); cur.clear(); }
            else cur += ch;
        }
        if (!cur.empty()) {          // the last operand may carry modifiers after a space
            std::istringstream ls(cur);
            std::string first;
            ls >> first;
            ops.push_back(first);
        }
    }
    const std::string &m = a.mn;
    const bool reads_dst = m.find("mac") != std::string::npos || m.find("_dpp") != std::string::npos;
    for (size_t k = 0; k < ops.size(); k++) {
        std::pair<int, int> r;
        if (parse_vreg(ops[k], r)) {
            a.vregs.push_back(r);
            if (k > 0 || reads_dst) a.vreads.push_back(r);
        } else if (parse_sreg(ops[k], r)) {
            a.sregs.push_back(r);
        }
    }
    a.dpp = m.find("_dpp") != std::string::npos;
    a.mfma = m.rfind("v_mfma", 0) == 0;
    const bool valu = m.rfind("v_", 0) == 0 && m.rfind("v_cmp", 0) != 0 && m.rfind("v_readlane", 0) != 0 &&
                      m.rfind("v_readfirstlane", 0) != 0;
    std::pair<int, int> r0;
    a.vdef0 = valu && !ops.empty() && parse_vreg(ops[0], r0);
    a.exec_valu_def = m.rfind("v_cmpx", 0) == 0;
    a.valu = m.rfind("v_", 0) == 0;
    for (const char *t : {"v_rcp_", "v_rsq_", "v_sqrt_", "v_exp_", "v_log_", "v_sin_", "v_cos_"})
        if (m.rfind(t, 0) == 0) a.trans = true;
    a.vmem = m.rfind("global_", 0) == 0 || m.rfind("buffer_", 0) == 0 || m.rfind("flat_", 0) == 0 ||
             m.rfind("scratch_", 0) == 0;
    if (a.valu) {                                   // SGPRs a VALU instruction writes
        std::pair<int, int> r;
        if (!ops.empty() && parse_sreg(ops[0], r)) a.sdefs.push_back(r);                      // v_cmp sdst, readlane
        if (m.find("_co_") != std::string::npos && ops.size() > 1 && parse_sreg(ops[1], r)) a.sdefs.push_back(r);
    }
    if (m == "s_nop") a.ws = 1 + (int)strtol(rest.c_str(), nullptr, 0);
    a.uncond = m == "s_branch" || m == "s_endpgm" || m.rfind("s_setpc", 0) == 0;
    return a;
}

bool overlap(const std::pair<int, int> &a, const std::pair<int, int> &b) {
    return a.first <= b.second && b.first <= a.second;
}

// Extra wait states instruction d needs: the maximum over every path into it
// (backward walk over fall-through and branch predecessors) of what a hazardous
// producer within its window demands.  `where` receives the worst producer.
int need_ws(const std::vector<Insn> &ins, const std::map<std::string, std::vector<size_t>> &preds_of,
            const std::map<size_t, std::string> &label_at, size_t d, std::string *where, int rules = R_DPP | R_TRANS) {
    const Insn &D = ins[d];
    int need = 0;
    std::vector<std::pair<size_t, int>> stack;
    auto push_preds = [&](size_t i, int ws) {
        if (i > 0 && !ins[i - 1].uncond) stack.push_back({i - 1, ws});
        auto lt = label_at.find(i);
        if (lt != label_at.end()) {
            auto it = preds_of.find(lt->second);
            if (it != preds_of.end())
                for (size_t p : it->second) stack.push_back({p, ws});
        }
    };
    push_preds(d, 0);
    int guard = 0;
    while (!stack.empty() && guard++ < 1 << 16) {
        auto [p, ws] = stack.back();
        stack.pop_back();
        const Insn &P = ins[p];
        int n = 0;
        if ((rules & R_DPP) && P.vdef0 && !P.vregs.empty())
            for (auto &u : D.vregs)
                if (overlap(P.vregs[0], u)) n = std::max(n, (P.mfma ? kMfmaWs : kDppVgprWs) - ws);
        if ((rules & R_DPP) && P.exec_valu_def) n = std::max(n, kDppExecWs - ws);
        if ((rules & R_TRANS) && P.trans && P.vdef0 && D.valu && !D.trans)
            for (auto &u : D.vreads)
                if (overlap(P.vregs[0], u)) n = std::max(n, kTransWs - ws);
        if ((rules & R_SGPR_VMEM) && D.vmem && P.valu)
            for (auto &sd : P.sdefs)
                for (auto &u : D.sregs)
                    if (overlap(sd, u)) n = std::max(n, kSgprVmemWs - ws);
        if (n > need) {
            need = n;
            if (where) *where = P.mn + " (" + std::to_string(ws) + " wait states before)";
        }
        if (ws + P.ws < kMaxWs) push_preds(p, ws + P.ws);
    }
    if (guard >= 1 << 16) need = std::max(need, kDppExecWs);   // walk cut short: be conservative
    return need;
}

}  // namespace

int asm_fixup(std::string &s, std::string *report) {
    // pass 1: instructions (with their line), labels, branches, inline-asm regions
    std::vector<std::string> lines;
    {
        std::istringstream in(s);
        std::string l;
        while (std::getline(in, l)) lines.push_back(l);
    }
    std::vector<Insn> ins;
    std::map<size_t, std::string> label_at;                 // instruction index -> (first) label before it
    std::map<std::string, size_t> pos_of;                   // label -> instruction index
    std::map<std::string, std::vector<size_t>> preds_of;    // canonical label -> branch instructions
    bool in_asm = false;
    for (size_t li = 0; li < lines.size(); li++) {
        std::string t = lines[li];
        const size_t c = t.find(';');
        const std::string cm = c == std::string::npos ? "" : t.substr(c);
        if (cm.rfind(";;#ASMSTART", 0) == 0) { in_asm = true; continue; }
        if (cm.rfind(";;#ASMEND", 0) == 0) { in_asm = false; continue; }
        if (c != std::string::npos) t = t.substr(0, c);
        const size_t b0 = t.find_first_not_of(" \t");
        if (b0 == std::string::npos) continue;
        t = t.substr(b0);
        while (!t.empty() && (t.back() == ' ' || t.back() == '\t' || t.back() == '\r')) t.pop_back();
        if (t.empty()) continue;
        if (t.back() == ':') {                              // a label
            const std::string name = t.substr(0, t.size() - 1);
            pos_of[name] = ins.size();
            label_at.emplace(ins.size(), name);             // several labels at one position: the first names it
            continue;
        }
        if (t[0] == '.') continue;                          // directive
        Insn a = parse_insn(t);
        a.line = li;
        a.dpp = a.dpp && in_asm;                            // ours to pad; the compiler pads its own
        if (a.mn == "s_branch" || a.mn.rfind("s_cbranch", 0) == 0) {
            std::istringstream ts(t);
            std::string mn, tgt;
            ts >> mn >> tgt;
            a.target = tgt;
        }
        ins.push_back(std::move(a));
    }
    for (size_t i = 0; i < ins.size(); i++)
        if (!ins[i].target.empty()) {
            auto it = pos_of.find(ins[i].target);
            if (it != pos_of.end()) preds_of[label_at[it->second]].push_back(i);
        }
    // pass 2: in program order, pad each DPP instruction of an asm region
    std::map<size_t, int> pad;                              // line -> s_nop count
    int sites = 0, states = 0;
    for (size_t d = 0; d < ins.size(); d++) {
        if (!ins[d].dpp) continue;
        const int n = need_ws(ins, preds_of, label_at, d, nullptr);
        if (n <= 0) continue;
        // the pad is an instruction in front of d: later walks see its wait states
        Insn nop;
        nop.mn = "s_nop";
        nop.ws = n;
        nop.line = ins[d].line;
        pad[ins[d].line] = n;
        sites++;
        states += n;
        ins.insert(ins.begin() + (long)d, nop);
        // shift positions >= d by one
        std::map<size_t, std::string> la;
        for (auto &kv : label_at) la[kv.first >= d ? kv.first + 1 : kv.first] = kv.second;
        label_at.swap(la);
        for (auto &kv : preds_of)
            for (auto &p : kv.second)
                if (p >= d) p++;
        d++;
    }
    if (!pad.empty()) {
        std::ostringstream o;
        for (size_t li = 0; li < lines.size(); li++) {
            auto it = pad.find(li);
            if (it != pad.end()) {
                int n = it->second;
                while (n > 0) {                             // s_nop k gives k + 1 wait states (k <= 15)
                    const int k = std::min(n, 16);
                    o << "\ts_nop " << (k - 1) << "    ; qpb_hazard: DPP operand wait states\n";
                    n -= k;
                }
            }
            o << lines[li] << '\n';
        }
        s = o.str();
    }
    if (report) *report = std::to_string(sites) + " DPP site(s) padded, " + std::to_string(states) + " wait states";
    return sites;
}

// ---- lane-partial code at a divergent region's join -------------------------------
// LLVM lowers `if (divergent) {...}` to
//     s_and_saveexec_b64 s[a:b], cond ; s_cbranch_execz J ; <then> ; J: s_or_b64 exec, exec, s[a:b]
// The register allocator treats J as the join block, i.e. code there runs for every
// lane -- but anything it places at J *before* the EXEC restore runs with the then
// region's EXEC (the skip path arrives with EXEC = 0).  The ROCm 7.2 backend does place
// live-range-split copies there, next to SGPR spills (v_writelane, which it counts as
// the block's prologue): e.g. `v_accvgpr_write_b32 a18, v124` parking a value every lane
// reads later, made only for the then-lanes.  The wide row kernel's memory-aperture
// violation was exactly that.  Moving those instructions to just after
// the restore gives them the semantics the allocator assumed.
namespace {

struct Ops {
    std::string mn;
    std::vector<std::pair<int, int>> defs, uses;   // v: 0..511, a: 512.., s: 1024.. (vcc 2024, exec 2026, m0 2028)
    bool mem = false, wait = false, valu_like = false, exec_def = false, trans = false, branch = false;
};

bool parse_reg(const std::string &tok, std::pair<int, int> &r) {
    size_t i = 0;
    while (i < tok.size() && (tok[i] == ' ' || tok[i] == '\t' || tok[i] == '-' || tok[i] == '|' || tok[i] == '!'))
        i++;
    const std::string t = tok.substr(i);
    if (t.rfind("vcc", 0) == 0) { r = {2024, 2025}; return true; }
    if (t.rfind("exec", 0) == 0) { r = {2026, 2027}; return true; }
    if (t.rfind("m0", 0) == 0) { r = {2028, 2028}; return true; }
    if (t.size() < 2) return false;
    const int base = t[0] == 'v' ? 0 : t[0] == 'a' ? 512 : t[0] == 's' ? 1024 : -1;
    if (base < 0) return false;
    int a = 0, b = 0;
    if (t[1] == '[') {
        if (sscanf(t.c_str() + 2, "%d:%d]", &a, &b) != 2) return false;
    } else if (isdigit((unsigned char)t[1])) {
        a = b = atoi(t.c_str() + 1);
    } else {
        return false;
    }
    r = {base + a, base + b};
    return true;
}

Ops parse_ops(const std::string &text) {
    Ops o;
    std::istringstream ts(text);
    ts >> o.mn;
    std::string rest;
    std::getline(ts, rest);
    std::vector<std::string> ops;
    std::string cur;
    for (char ch : rest) {
        if (ch == ',') { ops.push_back(cur); cur.clear(); }
        else cur += ch;
    }
    if (!cur.empty()) {
        std::istringstream ls(cur);
        std::string first;
        ls >> first;
        ops.push_back(first);
    }
    const std::string &m = o.mn;
    auto starts = [&](const char *p) { return m.rfind(p, 0) == 0; };
    const bool store = starts("global_store") || starts("buffer_store") || starts("scratch_store") ||
                       starts("flat_store") || starts("ds_write") || starts("global_atomic") ||
                       starts("buffer_atomic") || starts("ds_add") || starts("s_store");
    const bool nodef = store || starts("s_cmp") || starts("s_bitcmp") || starts("s_waitcnt") || starts("s_nop") ||
                       starts("s_branch") || starts("s_cbranch") || starts("s_endpgm") || starts("s_barrier") ||
                       starts("s_setprio") || starts("s_sleep");
    o.mem = starts("global_") || starts("buffer_") || starts("scratch_") || starts("flat_") || starts("ds_") ||
            starts("s_load") || starts("s_buffer_load") || starts("s_store");
    o.wait = starts("s_waitcnt");
    o.branch = starts("s_branch") || starts("s_cbranch") || starts("s_endpgm") || starts("s_setpc");
    o.valu_like = (starts("v_") || o.mem) && !starts("s_");
    for (const char *t : {"v_rcp_", "v_rsq_", "v_sqrt_", "v_exp_", "v_log_", "v_sin_", "v_cos_"})
        if (starts(t)) o.trans = true;
    const bool reads_dst = m.find("mac") != std::string::npos || m.find("_dpp") != std::string::npos ||
                           starts("v_writelane") || m.find("saveexec") != std::string::npos;
    for (size_t k = 0; k < ops.size(); k++) {
        std::pair<int, int> r;
        if (!parse_reg(ops[k], r)) continue;
        if (k == 0 && !nodef) {
            o.defs.push_back(r);
            if (reads_dst) o.uses.push_back(r);
        } else {
            o.uses.push_back(r);
        }
        if (k == 1 && m.find("_co_") != std::string::npos && r.first >= 1024) o.defs.push_back(r);   // carry-out
    }
    if (m.find("saveexec") != std::string::npos) { o.defs.push_back({2026, 2027}); o.uses.push_back({2026, 2027}); }
    for (auto &d : o.defs)
        if (d.first == 2026) o.exec_def = true;
    if (starts("v_cmpx")) o.exec_def = true;
    return o;
}

bool any_overlap(const std::vector<std::pair<int, int>> &a, const std::vector<std::pair<int, int>> &b) {
    for (auto &x : a)
        for (auto &y : b)
            if (x.first <= y.second && y.first <= x.second) return true;
    return false;
}

}  // namespace

int join_fixup(std::string &s, std::string *report) {
    std::vector<std::string> lines;
    {
        std::istringstream in(s);
        std::string l;
        while (std::getline(in, l)) lines.push_back(l);
    }
    auto code_of = [&](size_t li) -> std::string {      // instruction text, "" for non-instructions
        std::string t = lines[li];
        const size_t c = t.find(';');
        if (c != std::string::npos) t = t.substr(0, c);
        const size_t b0 = t.find_first_not_of(" \t");
        if (b0 == std::string::npos) return "";
        t = t.substr(b0);
        while (!t.empty() && (t.back() == ' ' || t.back() == '\t' || t.back() == '\r')) t.pop_back();
        if (t.empty() || t[0] == '.' || t.back() == ':') return "";
        return t;
    };
    auto label_of = [&](size_t li) -> std::string {
        std::string t = lines[li];
        const size_t c = t.find(';');
        if (c != std::string::npos) t = t.substr(0, c);
        while (!t.empty() && (t.back() == ' ' || t.back() == '\t' || t.back() == '\r')) t.pop_back();
        if (!t.empty() && t.back() == ':' && t[0] != ' ' && t[0] != '\t') return t.substr(0, t.size() - 1);
        return "";
    };
    std::map<std::string, size_t> label_line;
    for (size_t li = 0; li < lines.size(); li++) {
        const std::string lb = label_of(li);
        if (!lb.empty()) label_line[lb] = li;
    }
    struct Move { size_t restore; std::vector<size_t> moved; int pad; };
    std::map<size_t, Move> moves;                            // keyed by the restore line
    int fixed = 0, unfixed = 0, insns = 0;
    std::ostringstream why;
    for (size_t li = 0; li < lines.size(); li++) {
        const std::string t = code_of(li);
        if (t.rfind("s_cbranch_execz", 0) != 0) continue;
        std::istringstream ts(t);
        std::string mn, tgt;
        ts >> mn >> tgt;
        auto it = label_line.find(tgt);
        if (it == label_line.end()) continue;
        std::vector<size_t> cand, other;                      // lines before the restore
        size_t restore = 0;
        bool ok = true;
        for (size_t k = it->second + 1; k < lines.size(); k++) {
            if (!label_of(k).empty()) { ok = false; break; }  // another block starts: not this pattern
            const std::string c = code_of(k);
            if (c.empty()) continue;
            const Ops o = parse_ops(c);
            if (o.exec_def) {
                if (o.mn == "s_or_b64" && c.find("exec, exec,") != std::string::npos) restore = k;
                else ok = false;
                break;
            }
            if (o.branch) { ok = false; break; }
            const bool lane_masked = o.valu_like && o.mn.rfind("v_writelane", 0) != 0 &&
                                     o.mn.rfind("v_readlane", 0) != 0 && o.mn.rfind("v_readfirstlane", 0) != 0 &&
                                     o.mn.rfind("v_cmp", 0) != 0;
            (lane_masked ? cand : other).push_back(k);
        }
        if (!ok || !restore || cand.empty()) continue;
        // may each candidate move past the instructions after it (and the restore)?
        bool movable = true;
        for (size_t a : cand) {
            const Ops A = parse_ops(code_of(a));
            if (A.trans) movable = false;
            std::vector<size_t> past;
            for (size_t b : other)
                if (b > a) past.push_back(b);
            past.push_back(restore);
            for (size_t b : past) {
                const Ops Bo = parse_ops(code_of(b));
                if (any_overlap(A.uses, Bo.defs) || any_overlap(A.defs, Bo.uses) || any_overlap(A.defs, Bo.defs))
                    movable = false;
                if (A.mem && (Bo.mem || Bo.wait)) movable = false;
            }
        }
        if (!movable) {
            unfixed++;
            why << "join " << tgt << " (line " << it->second + 1 << ") not movable; ";
            continue;
        }
        int npast = 1;                                       // the restore itself
        for (size_t b : other)
            if (b > cand.front()) npast++;
        moves[restore] = Move{restore, cand, std::min(npast, 16)};
        fixed++;
        insns += (int)cand.size();
    }
    if (!moves.empty()) {
        std::map<size_t, bool> drop;
        for (auto &kv : moves)
            for (size_t a : kv.second.moved) drop[a] = true;
        std::ostringstream o;
        for (size_t li = 0; li < lines.size(); li++) {
            if (drop.count(li)) continue;
            o << lines[li] << '\n';
            auto mv = moves.find(li);
            if (mv != moves.end()) {
                for (size_t a : mv->second.moved)
                    o << lines[a] << "    ; qpb_hazard: moved past the EXEC restore (join_fixup)\n";
                // keep every moved result at least as far from its readers as before
                o << "\ts_nop " << (mv->second.pad - 1) << "    ; qpb_hazard: join_fixup distance\n";
            }
        }
        s = o.str();
    }
    if (report)
        *report = std::to_string(fixed) + " join(s) repaired (" + std::to_string(insns) + " instruction(s) moved past "
                  "the EXEC restore)" + (unfixed ? ", " + std::to_string(unfixed) + " not movable: " + why.str() : "");
    return unfixed ? -unfixed : fixed;
}

int audit_disassembly(const std::string &dis, std::string *report) {
    std::vector<Insn> ins;
    std::map<size_t, std::string> label_at;
    std::map<std::string, std::vector<size_t>> preds_of;
    std::map<uint64_t, size_t> at;
    std::vector<std::pair<size_t, uint64_t>> branches;
    std::vector<std::string> texts;
    uint64_t fbase = 0;
    std::istringstream in(dis);
    std::string line;
    while (std::getline(in, line)) {
        if (!line.empty() && isxdigit((unsigned char)line[0]) && line.find(">:") != std::string::npos) {
            fbase = strtoull(line.c_str(), nullptr, 16);           // "0000000000001d00 <name>:"
            continue;
        }
        if (line.empty() || line[0] != '\t') continue;
        const size_t cm = line.find("// ");
        if (cm == std::string::npos) continue;
        const uint64_t addr = strtoull(line.c_str() + cm + 3, nullptr, 16);
        Insn a = parse_insn(line.substr(1, cm - 1));
        if (a.mn == "s_branch" || a.mn.rfind("s_cbranch", 0) == 0) {
            const size_t lt = line.find('<', cm);
            if (lt != std::string::npos) {
                const size_t plus = line.find("+0x", lt);
                branches.push_back({ins.size(), fbase + (plus != std::string::npos
                                                            ? strtoull(line.c_str() + plus + 3, nullptr, 16) : 0)});
            }
        }
        at[addr] = ins.size();
        ins.push_back(std::move(a));
        texts.push_back(line.substr(1, cm - 1));
    }
    if (ins.empty()) {
        *report = "empty disassembly";
        return -1;
    }
    for (auto &[i, tgt] : branches) {
        auto it = at.find(tgt);
        if (it == at.end()) continue;
        const std::string name = "@" + std::to_string(it->second);
        label_at[it->second] = name;
        preds_of[name].push_back(i);
    }
    int hazards = 0, other = 0;
    std::ostringstream rep;
    for (size_t d = 0; d < ins.size(); d++) {
        const Insn &D = ins[d];
        int rules = 0;
        if (D.dpp) rules |= R_DPP;
        if (D.valu && !D.trans) rules |= R_TRANS;
        if (D.vmem) rules |= R_SGPR_VMEM;
        if (!rules) continue;
        std::string where;
        const int n = need_ws(ins, preds_of, label_at, d, &where, rules);
        if (n <= 0) continue;
        if (D.dpp) hazards++;
        else other++;
        if (hazards + other <= 8) rep << D.mn << " needs " << n << " more wait state(s) after " << where << "; ";
    }
    // lane-partial code at a join (join_fixup's pattern): a lane-masked instruction
    // between an s_cbranch_execz target and the EXEC restore that follows it
    int joins = 0;
    for (auto &[i, tgt] : branches) {
        if (ins[i].mn != "s_cbranch_execz") continue;
        auto it = at.find(tgt);
        if (it == at.end()) continue;
        int masked = 0;
        for (size_t k = it->second; k < ins.size(); k++) {
            if (k > it->second && label_at.count(k)) break;
            const Ops o = parse_ops(texts[k]);
            if (o.exec_def) {
                if (masked && o.mn == "s_or_b64" && texts[k].find("exec, exec,") != std::string::npos) {
                    joins++;
                    if (hazards + other + joins <= 8)
                        rep << masked << " lane-masked instruction(s) before the EXEC restore at join +" << k << "; ";
                }
                break;
            }
            if (o.branch) break;
            if (o.valu_like && o.mn.rfind("v_writelane", 0) != 0 && o.mn.rfind("v_readlane", 0) != 0 &&
                o.mn.rfind("v_readfirstlane", 0) != 0 && o.mn.rfind("v_cmp", 0) != 0)
                masked++;
        }
    }
    *report = (hazards || other || joins)
                  ? std::to_string(hazards) + " DPP hazard(s), " + std::to_string(other) +
                        " trans-forwarding / SGPR->VMEM hazard(s), " + std::to_string(joins) +
                        " lane-partial join(s): " + rep.str()
                  : "clean (DPP, trans forwarding, VALU SGPR -> VMEM, EXEC-restore joins)";
    return (hazards || other || joins) ? 0 : 1;
}

}  // namespace qpb
