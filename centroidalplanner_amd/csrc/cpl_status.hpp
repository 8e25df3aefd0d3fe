// cpl_status.hpp — error plumbing of the C-ABI (status codes + thread-local last message).
#pragma once

#include <cstdint>
#include <string>

#include "../../include/cpl_mi355x.h"

namespace cpl {
int32_t fail(int32_t status, const std::string& msg);
int32_t validate_desc(const cpl_problem_desc* d);
}  // namespace cpl
