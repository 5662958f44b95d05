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

int audit_disassembly(const std::string &dis, std::string *report) {
    std::vector<Insn> ins;
    std::map<size_t, std::string> label_at;
    std::map<std::string, std::vector<size_t>> preds_of;
    std::map<uint64_t, size_t> at;
    std::vector<std::pair<size_t, uint64_t>> branches;
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
    *report = (hazards || other) ? std::to_string(hazards) + " DPP hazard(s), " + std::to_string(other) +
                                       " trans-forwarding / SGPR->VMEM hazard(s): " + rep.str()
                                 : "clean (DPP, trans forwarding, VALU SGPR -> VMEM)";
    return (hazards || other) ? 0 : 1;
}

}  // namespace qpb
