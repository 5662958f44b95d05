// qpb_hazard.hpp -- wait states for DPP inline asm (qpb_hazard.cpp).
#pragma once

#include <string>

namespace qpb {
// Pad every DPP instruction inside an inline-asm region of the assembly text s
// (clang -S output) with the s_nop its VGPR / EXEC producers require on every
// path into it.  Returns the number of padded sites; *report summarises.
int asm_fixup(std::string &s, std::string *report);
// Move lane-masked instructions the register allocator placed between a divergent
// region's skip target (s_cbranch_execz) and its EXEC restore (s_or_b64 exec, exec, ..)
// to just after the restore.  Returns the number of repaired joins, or -k when k joins
// could not be repaired (*report names them).
int join_fixup(std::string &s, std::string *report);
// Check a disassembled code object (llvm-objdump -d): 1 clean, 0 hazard found
// (*report says where), -1 could not audit.
int audit_disassembly(const std::string &dis, std::string *report);
}  // namespace qpb
