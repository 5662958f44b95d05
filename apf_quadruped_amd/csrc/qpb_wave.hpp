// qpb_wave.hpp -- wave-cooperative kernel generator (one wavefront per QP).
#pragma once

#include <string>

#include "qpb_plan.hpp"

namespace qpb {
// Can the plan run on the wave kernel?  (n, m, p <= 64; no empty G row.)
bool wave_eligible(const Plan &pl, std::string *why);
// Full hiprtc source; the kernel name is returned through name_out.
std::string generate_wave_kernel(const Plan &pl, int wg, std::string *name_out);
}  // namespace qpb
