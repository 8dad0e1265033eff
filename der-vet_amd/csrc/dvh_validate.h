// dvh_validate.h -- host-side validation of a dvh_lp (dvh_validate.cpp); no HIP dependency.
#pragma once
#include <string>

#include "../../include/dervet_hip.h"

namespace dvh {
// "" when the window is well formed; otherwise the error message dvh_last_error reports (sizes, null arrays, CSR
// row pointers monotone from 0 to nnz, column indices in range, no duplicate column in a row, finite matrix values,
// right-hand sides and objective, no NaN bound, l < +inf and u > -inf; crossed finite bounds are a valid, infeasible
// window).  k: the window's index in the batch, for the message.
std::string validate_lp(const dvh_lp& lp, int k);
}  // namespace dvh
