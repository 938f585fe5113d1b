// matvec_ks4.hip — instantiations of the matvec kernels for K split 4 (one translation unit per
// split so the kernel variants compile in parallel; the kernels are in matvec_impl.h).
#include "matvec_impl.h"

namespace ghip {
int matvec_dispatch_ks4(int wtype, int pro, int epi, const mv_args &a, int g, hipStream_t s) {
    if (wtype == T_Q4_0) return dispatch_pro<T_Q4_0, 4>(pro, epi, a, g, s);
    if (wtype == T_Q8_0) return dispatch_pro<T_Q8_0, 4>(pro, epi, a, g, s);
    set_error("matvec: unsupported weight type");
    return -1;
}
}  // namespace ghip
