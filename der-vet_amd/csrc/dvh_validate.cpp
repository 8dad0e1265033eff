// dvh_validate.cpp -- validation of a caller's host LP (the untrusted input of dvh_solve_batch, include/dervet_hip.h)
// before anything is packed or copied to the device.  Plain C++ with no HIP dependency, so the same code also runs in
// the CPU restatement (oracle/cpu_pdhg.cpp) and in its AddressSanitizer / UBSan build (oracle/abi_sanitize.cpp,
// tests/test_sanitize.py), which feeds it malformed CSR.
#include "dvh_validate.h"

#include <cmath>
#include <cstdint>
#include <cstdio>

namespace dvh {

std::string validate_lp(const dvh_lp& lp, int k) {
  char buf[256];
  if (lp.n <= 0 || lp.m_eq < 0 || lp.m_ineq < 0 || lp.nnz < 0 || (int64_t)lp.m_eq + lp.m_ineq > INT32_MAX - 1) {
    snprintf(buf, sizeof buf, "window %d: invalid sizes n=%d m_eq=%d m_ineq=%d nnz=%d", k, lp.n, lp.m_eq, lp.m_ineq,
             lp.nnz);
    return buf;
  }
  const int m = lp.m_eq + lp.m_ineq;
  if (!lp.indptr || (lp.nnz > 0 && (!lp.indices || !lp.data)) || !lp.c || (m > 0 && !lp.q) || !lp.l || !lp.u) {
    snprintf(buf, sizeof buf, "window %d: null array", k);
    return buf;
  }
  if (lp.indptr[0] != 0 || lp.indptr[m] != lp.nnz) {
    snprintf(buf, sizeof buf, "window %d: indptr[0] must be 0 and indptr[m] == nnz", k);
    return buf;
  }
  for (int i = 0; i < m; ++i)
    if (lp.indptr[i + 1] < lp.indptr[i]) {
      snprintf(buf, sizeof buf, "window %d: indptr not monotone at row %d", k, i);
      return buf;
    }
  for (int p = 0; p < lp.nnz; ++p) {
    if (lp.indices[p] < 0 || lp.indices[p] >= lp.n) {
      snprintf(buf, sizeof buf, "window %d: column index %d out of range at nnz %d", k, lp.indices[p], p);
      return buf;
    }
    if (!std::isfinite(lp.data[p])) {
      snprintf(buf, sizeof buf, "window %d: non-finite matrix value at nnz %d", k, p);
      return buf;
    }
  }
  for (int i = 0; i < m; ++i) {
    // duplicate column within a row makes the transpose ambiguous for nothing; reject
    for (int p = lp.indptr[i] + 1; p < lp.indptr[i + 1]; ++p)
      for (int r = lp.indptr[i]; r < p; ++r)
        if (lp.indices[r] == lp.indices[p]) {
          snprintf(buf, sizeof buf, "window %d: duplicate column %d in row %d", k, lp.indices[p], i);
          return buf;
        }
    if (!std::isfinite(lp.q[i])) {
      snprintf(buf, sizeof buf, "window %d: non-finite rhs at row %d", k, i);
      return buf;
    }
  }
  for (int j = 0; j < lp.n; ++j) {
    // crossed finite bounds (l > u) are a valid, infeasible window: status PRIMAL_INFEASIBLE (setup kernel)
    if (!std::isfinite(lp.c[j]) || std::isnan(lp.l[j]) || std::isnan(lp.u[j]) || lp.l[j] == INFINITY ||
        lp.u[j] == -INFINITY) {
      snprintf(buf, sizeof buf, "window %d: invalid objective or bounds at variable %d", k, j);
      return buf;
    }
  }
  if (!std::isfinite(lp.c0)) {
    snprintf(buf, sizeof buf, "window %d: non-finite c0", k);
    return buf;
  }
  return "";
}

}  // namespace dvh
