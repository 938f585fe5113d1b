// matvec.hip — launch entry of the decode matvec (kernels: matvec_impl.h, instantiated per K split
// in matvec_ks{1,2,4,8}.hip).
#include "matvec_impl.h"

namespace ghip {
int matvec_dispatch_ks1(int wtype, int pro, int epi, const mv_args &a, int g, hipStream_t s);
int matvec_dispatch_ks2(int wtype, int pro, int epi, const mv_args &a, int g, hipStream_t s);
int matvec_dispatch_ks4(int wtype, int pro, int epi, const mv_args &a, int g, hipStream_t s);
int matvec_dispatch_ks8(int wtype, int pro, int epi, const mv_args &a, int g, hipStream_t s);
int matvec_dispatch_rr(int wtype, int pro, int epi, const mv_args &a, hipStream_t s);

size_t matvec_lds_bytes(int wtype, int ks, int64_t n_bt, int64_t seg) {
    const bool nsa = ks != 8;  // as launch_t
    if (wtype == T_Q4_0) return nsa ? make_lds_map<T_Q4_0, true>(ks, n_bt, seg).total : make_lds_map<T_Q4_0, false>(ks, n_bt, seg).total;
    return make_lds_map<T_Q8_0, true>(ks, n_bt, seg).total;
}

int launch_matvec(int wtype, int ks, int pro, int epi, const mv_args &a, int grid_x, hipStream_t s) {
    if (a.n_rt <= 0 || a.n_bt <= 0) return 0;
    if (grid_x <= 0) {
        set_error("matvec: grid_x <= 0");
        return -1;
    }
    // the tiled weight image: n_bt block tiles of BT blocks cover the nb = K/32 blocks, the padded
    // tail (< BT blocks) is zero-filled in the activation image
    const int64_t bt = wtype == T_Q4_0 ? wfmt<T_Q4_0>::BT : wfmt<T_Q8_0>::BT;
    if (a.nb <= 0 || a.n_bt != (a.nb + bt - 1) / bt || a.n_rt != (a.rows + 7) / 8 || a.ncols <= 0) {
        set_error("matvec: shape mismatch (n_bt must be ceil(K/32 / BT), n_rt ceil(rows / 8), ncols > 0)");
        return -1;
    }
    if (wtype != T_Q4_0 && wtype != T_Q8_0) {
        set_error("matvec: weight type must be Q4_0 or Q8_0");
        return -1;
    }
    int r = -1;
    switch (ks) {
        case 1: r = matvec_dispatch_ks1(wtype, pro, epi, a, grid_x, s); break;
        case 2: r = matvec_dispatch_ks2(wtype, pro, epi, a, grid_x, s); break;
        case 4: r = matvec_dispatch_ks4(wtype, pro, epi, a, grid_x, s); break;
        case 8: r = matvec_dispatch_ks8(wtype, pro, epi, a, grid_x, s); break;
        case KS_RR: r = matvec_dispatch_rr(wtype, pro, epi, a, s); break;  // grid = one workgroup per row tile
        default: set_error("matvec: unsupported KS");
    }
    if (r != 0 && last_error().empty()) set_error("matvec: bad (ks, pro, epi) combination");
    return r;
}

}  // namespace ghip
