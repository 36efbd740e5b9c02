#ifndef GEEPS_AMD_CHECK_HPP_
#define GEEPS_AMD_CHECK_HPP_

// Fail-loudly helpers for libgeeps.  The reference aborts through glog CHECK /
// CUDA_CHECK (src/common/gpu-util/device_alternate.hpp:16-28); libgeeps keeps
// that contract without glog: a violated invariant or a failed C-ABI call
// prints file:line and the message, then aborts.

#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>

#include "gp_reduce.h"

namespace geeps {

[[noreturn]] inline void die(const char *file, int line, const std::string &msg) {
  std::fprintf(stderr, "libgeeps FATAL %s:%d: %s\n", file, line, msg.c_str());
  std::fflush(stderr);
  std::abort();
}

}  // namespace geeps

#define GP_CHECK(cond)                                                        \
  do {                                                                        \
    if (!(cond)) ::geeps::die(__FILE__, __LINE__, "check failed: " #cond);   \
  } while (0)

#define GP_CHECK_MSG(cond, what)                                              \
  do {                                                                        \
    if (!(cond)) {                                                            \
      std::ostringstream os_;                                                 \
      os_ << "check failed: " #cond " — " << what;                            \
      ::geeps::die(__FILE__, __LINE__, os_.str());                            \
    }                                                                         \
  } while (0)

#define GP_CHECK_OP(a, op, b)                                                 \
  do {                                                                        \
    const auto va_ = (a);                                                     \
    const auto vb_ = (b);                                                     \
    if (!(va_ op vb_)) {                                                      \
      std::ostringstream os_;                                                 \
      os_ << "check failed: " #a " " #op " " #b " (" << va_ << " vs " << vb_  \
          << ")";                                                             \
      ::geeps::die(__FILE__, __LINE__, os_.str());                            \
    }                                                                         \
  } while (0)

#define GP_CHECK_EQ(a, b) GP_CHECK_OP(a, ==, b)
#define GP_CHECK_LT(a, b) GP_CHECK_OP(a, <, b)
#define GP_CHECK_LE(a, b) GP_CHECK_OP(a, <=, b)
#define GP_CHECK_GE(a, b) GP_CHECK_OP(a, >=, b)

// A C-ABI call (include/gp_reduce.h) that must succeed.
#define GP_CALL(expr)                                                         \
  do {                                                                        \
    const int rc_ = (expr);                                                   \
    if (rc_ != GP_OK) {                                                       \
      std::ostringstream os_;                                                 \
      os_ << #expr " -> status " << rc_ << ": " << gp_last_error();           \
      ::geeps::die(__FILE__, __LINE__, os_.str());                            \
    }                                                                         \
  } while (0)

#endif  // GEEPS_AMD_CHECK_HPP_
