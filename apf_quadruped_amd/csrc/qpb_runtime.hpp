// qpb_runtime.hpp -- internals shared by the batched C ABI and the qpSWIFT drop-in.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "qpb_codegen.hpp"
#include "qpb_plan.hpp"

struct qpb_plan {
    qpb::Plan pl;
    qpb::GenOptions gen;
    std::string kname;
    std::shared_ptr<std::vector<char>> code;
};

namespace qpb {
int compile_plan(qpb_plan *plan);
int set_error(int code, const char *msg);
}  // namespace qpb
