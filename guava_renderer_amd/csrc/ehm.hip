// ehm.hip -- EHM.forward (modules/ehm/EHM.py:36-156 of the reference) as one host call
// (gsr_ehm_forward, include/gsr_deform.h).
//
// The reference's forward is torch glue around two lbs() calls: it concatenates / zero-pads / expands
// the parameter dicts into coefficient rows (EHM.py:41-48, :94-112), runs the FLAME head lbs, the body
// template's blend shapes and joints, splices the head (with eyelids and head scale) into the body
// template and runs the body lbs_wobeta.  Here the row assembly is one launch of k_ehm_pack (its
// table built on the host from the parameter descriptors) and the rest are the gsr_lbs_sp /
// gsr_blend_joints_sp / gsr_splice_head launches, all issued from C: a single-frame call crosses the
// FFI once and builds no tables in Python (the per-frame drop-in loop's deform was host-bound on
// that).
#include <algorithm>
#include <string>
#include <vector>

#include "../../include/gsr.h"
#include "../../include/gsr_deform.h"
#include "deform_internal.h"
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kEhmMaxSegments = 24;
struct EhmPackTable {
    GsrRowSegment seg[kEhmMaxSegments];
};

// one workgroup per (segment, frame), as k_pack_rows
__global__ __launch_bounds__(256) void k_ehm_pack(EhmPackTable t) {
    const GsrRowSegment sg = t.seg[blockIdx.x];
    const int b = blockIdx.y;
    for (int c = threadIdx.x; c < sg.width; c += 256)
        sg.dst[b * sg.dst_stride + c] = sg.src ? sg.src[b * sg.src_stride + c] : 0.f;
}

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

struct EhmArena {
    float *betas_h, *pose_h, *betas_b, *pose_b, *hscale, *eyelid, *joff;
    float *hv, *hj, *vt, *tj;
    char *ws_h, *ws_b;
};

size_t carve_ehm(char* base, const GsrEhm& e, int B, EhmArena* a) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* p = base ? base + off : nullptr;
        off += al(bytes);
        return p;
    };
    auto tf = [&](size_t n) { return reinterpret_cast<float*>(take(sizeof(float) * n)); };
    const size_t b = (size_t)B;
    EhmArena t;
    t.betas_h = tf(b * e.flame.NB);
    t.pose_h = tf(b * 3 * e.flame.J);
    t.betas_b = tf(b * e.body.NB);
    t.pose_b = tf(b * 3 * e.body.J);
    t.hscale = tf(b * 3);
    t.eyelid = tf(b * 2);
    t.joff = tf(b * 3 * e.body.J);
    t.hv = tf(b * e.flame.V * 3);
    t.hj = tf(b * e.flame.J * 3);
    t.vt = tf(b * e.body.V * 3);
    t.tj = tf(b * e.body.J * 3);
    t.ws_h = take(gsr_lbs_workspace_bytes(B, e.flame.V, e.flame.J, e.flame.NB));
    t.ws_b = take(gsr_lbs_workspace_bytes(B, e.body.V, e.body.J, 0));
    if (a) *a = t;
    return off;
}

// The row table of one destination block [B][width]: its copies plus a zero segment for every column
// run no copy covers (the reference's zeros); copies must not overlap.
struct Copy {
    int col, width;
    const float* src;
    int64_t src_stride;
};
int add_block(std::vector<GsrRowSegment>& tab, float* dst, int width, std::vector<Copy> cp, const char* what) {
    std::sort(cp.begin(), cp.end(), [](const Copy& x, const Copy& y) { return x.col < y.col; });
    int c = 0;
    for (const Copy& k : cp) {
        if (k.width <= 0) continue;
        if (k.col < c || k.col + k.width > width)
            return api_fail(GSR_ERR_ARG, (std::string("gsr_ehm_forward: ") + what +
                                          ": a parameter does not fit its coefficient columns").c_str());
        if (k.col > c) tab.push_back(GsrRowSegment{nullptr, dst + c, 0, width, k.col - c, 0});
        tab.push_back(GsrRowSegment{k.src, dst + k.col, k.src_stride, width, k.width, 0});
        c = k.col + k.width;
    }
    if (c < width) tab.push_back(GsrRowSegment{nullptr, dst + c, 0, width, width - c, 0});
    return 0;
}

int check_model(const GsrEhmModel& m, const char* who) {
    if (m.V <= 0 || m.J < 1 || m.J > GSR_LBS_MAX_JOINTS || m.NB < 0 || !m.v_template || !m.J_regressor ||
        !m.parents_host || !m.lbs_weights_t || (m.J > 1 && !m.posedirs) || (m.NB > 0 && !m.shapedirs_t))
        return api_fail(GSR_ERR_ARG, (std::string("gsr_ehm_forward: bad ") + who + " model").c_str());
    return 0;
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_ehm_workspace_bytes(const GsrEhm* ehm, int B) {
    if (!ehm || B <= 0) return 0;
    return carve_ehm(nullptr, *ehm, B, nullptr);
}

int gsr_ehm_forward(const GsrEhm* ehm, int B, const GsrEhmParam* params, const GsrEhmOutputs* out,
                    char* workspace, void* stream) {
    if (!ehm || !params || !out || !out->vertices || !workspace || B <= 0)
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: null argument or B <= 0");
    const GsrEhm& e = *ehm;
    if (int rc = check_model(e.flame, "FLAME")) return rc;
    if (int rc = check_model(e.body, "body")) return rc;
    if (e.N_head != e.flame.V || !e.head_index)
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: N_head must equal the FLAME vertex count, with head_index");
    for (int i = 0; i < GSR_EHM_NPARAM; i++) {
        const GsrEhmParam& p = params[i];
        if (p.p && (p.width <= 0 || (p.row_stride != 0 && p.row_stride < p.width)))
            return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: a parameter has a bad width or row stride");
    }
    if (!params[GSR_EHM_FLAME_SHAPE].p || !params[GSR_EHM_BODY_SHAPE].p || !params[GSR_EHM_BODY_EXP].p ||
        !params[GSR_EHM_BODY_LHAND].p || !params[GSR_EHM_BODY_RHAND].p)
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: FLAME shape, body shape / exp and both hand poses are required");
    const GsrEhmParam& eyel = params[GSR_EHM_FLAME_EYELID];
    const GsrEhmParam& hsc = params[GSR_EHM_BODY_HEAD_SCALE];
    const GsrEhmParam& jof = params[GSR_EHM_BODY_JOINTS_OFFSET];
    if ((eyel.p && eyel.width != 2) || (hsc.p && hsc.width != 3) || (jof.p && jof.width != 3 * e.body.J))
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: eyelid_params must be 2 wide, head_scale 3, joints_offset 3J");
    if ((eyel.p && (!e.l_eyelid || !e.r_eyelid)))
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: eyelid_params need both eyelid bases");
    const GsrEhmParam& gp = params[GSR_EHM_BODY_GLOBAL];
    const GsrEhmParam& bpo = params[GSR_EHM_BODY_POSE];
    // (EHM.py:107-114 concatenates them as they are: another width would misalign the pose row)
    if ((gp.p && gp.width != 3) || (bpo.p && bpo.width != 63))
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: global_pose must be 3 columns wide, body_pose 63");

    EhmArena a;
    carve_ehm(workspace, e, B, &a);
    const int Vh = e.flame.V, Jh = e.flame.J, NBh = e.flame.NB;
    const int Vb = e.body.V, Jb = e.body.J, NBb = e.body.NB;
    // the coefficient rows (EHM.py:41-48 FLAME betas / pose; :94-112 body betas / pose)
    std::vector<GsrRowSegment> tab;
    auto cp = [&](int slot, int col, int width) {
        const GsrEhmParam& p = params[slot];
        return Copy{col, p.p ? width : 0, p.p, p.row_stride};
    };
    const int ws_h = params[GSR_EHM_FLAME_SHAPE].width;
    const int w_exp = params[GSR_EHM_BODY_EXP].width;
    const int n_shape = NBb - w_exp;
    if (n_shape < 0) return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: exp is wider than the body blend");
    // FLAME betas (EHM.py:53-62): shape_params zero-padded to flame.n_shape, then the expression, so
    // the expression starts at n_shape = NB - its width whatever the shape width passed
    const int we_h = params[GSR_EHM_FLAME_EXPR].p ? params[GSR_EHM_FLAME_EXPR].width : 0;
    const int n_shape_h = NBh - we_h;
    if (n_shape_h < 0 || ws_h > n_shape_h)
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: FLAME betas: shape + expression wider than the FLAME blend");
    if (int rc = add_block(tab, a.betas_h, NBh,
                           {cp(GSR_EHM_FLAME_SHAPE, 0, ws_h), cp(GSR_EHM_FLAME_EXPR, n_shape_h, we_h)},
                           "FLAME betas"))
        return rc;
    if (int rc = add_block(tab, a.pose_h, 3 * Jh,
                           {cp(GSR_EHM_FLAME_JAW, 6, params[GSR_EHM_FLAME_JAW].width),
                            cp(GSR_EHM_FLAME_EYES, 9, params[GSR_EHM_FLAME_EYES].width)}, "FLAME pose"))
        return rc;
    if (int rc = add_block(tab, a.betas_b, NBb,
                           {cp(GSR_EHM_BODY_SHAPE, 0, std::min(n_shape, params[GSR_EHM_BODY_SHAPE].width)),
                            cp(GSR_EHM_BODY_EXP, n_shape, w_exp)}, "body betas"))
        return rc;
    if (int rc = add_block(tab, a.pose_b, 3 * Jb,
                           {cp(GSR_EHM_BODY_GLOBAL, 0, 3), cp(GSR_EHM_BODY_POSE, 3, 63),
                            cp(GSR_EHM_BODY_LHAND, 75, params[GSR_EHM_BODY_LHAND].width),
                            cp(GSR_EHM_BODY_RHAND, 120, params[GSR_EHM_BODY_RHAND].width)}, "body pose"))
        return rc;
    // eyelids / head scale / joint offsets are read per frame at their natural row width: passed as
    // they are when that holds (or for one frame), else expanded into the workspace
    auto direct = [&](const GsrEhmParam& p) { return p.row_stride == p.width || B == 1; };
    const float* eyelid = eyel.p;
    if (eyel.p && !direct(eyel)) {
        tab.push_back(GsrRowSegment{eyel.p, a.eyelid, eyel.row_stride, 2, 2, 0});
        eyelid = a.eyelid;
    }
    const float* hscale = hsc.p;
    if (hsc.p && !direct(hsc)) {
        tab.push_back(GsrRowSegment{hsc.p, a.hscale, hsc.row_stride, 3, 3, 0});
        hscale = a.hscale;
    }
    const float* joff = jof.p;
    if (jof.p && !direct(jof)) {
        tab.push_back(GsrRowSegment{jof.p, a.joff, jof.row_stride, 3 * Jb, 3 * Jb, 0});
        joff = a.joff;
    }
    if (tab.size() > (size_t)kEhmMaxSegments)
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: too many coefficient segments");
    EhmPackTable t;
    for (size_t i = 0; i < tab.size(); i++) {
        if (tab[i].width > 4096) return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: coefficient row too wide");
        t.seg[i] = tab[i];
    }
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_ehm_pack, dim3((unsigned)tab.size(), B), dim3(256), 0, s, t);
    if (hipError_t err = hipGetLastError(); err != hipSuccess)
        return api_fail(GSR_ERR_HIP, (std::string("ehm_pack: ") + hipGetErrorString(err)).c_str());

    // FLAME head lbs (EHM.py:67-70): posed joints, and the head vertices unless the skinning is fused
    // into the splice below (ELL weights; GSR_EHM_SKIN_SPLICE=0: separate, A/B)
    static const bool skin_splice_on = tune_env("GSR_EHM_SKIN_SPLICE", 1) != 0;
    const bool fuse = skin_splice_on && e.flame.sparse && e.flame.sparse->skin_k > 0;
    // one frame: the body's shape blend (independent of the head) rides in the head blend's launch
    Blend1Job body_shape{};
    static const bool pair_on = tune_env("GSR_EHM_PAIR", 1) != 0;  // 0: separate launches (A/B)
    const bool pair = pair_on && B == 1 && blend_tiled1_applies(1, NBb, 0, nullptr, e.body.sparse);
    if (pair)
        body_shape = blend1_job(Vb * 3, NBb, 0, e.body.v_template, a.betas_b, nullptr, a.vt, nullptr, e.body.sparse,
                                nullptr, 1);
    bool body_blended = false;
    int rc = lbs_run(B, Vh, Jh, NBh, e.flame.v_template, 0, a.betas_h, e.flame.shapedirs_t, a.pose_h, 1,
                     e.flame.posedirs, e.flame.J_regressor, e.flame.parents_host, e.flame.lbs_weights_t, nullptr,
                     a.hv, a.hj, nullptr, nullptr, nullptr, nullptr, a.ws_h, e.flame.sparse, stream, !fuse,
                     pair ? &body_shape : nullptr, &body_blended);
    if (rc) return rc;
    // body template: blend shapes + joints (+ offset) (EHM.py:114-118)
    rc = blend_joints_run(B, Vb, Jb, NBb, e.body.v_template, 0, a.betas_b, e.body.shapedirs_t, e.body.J_regressor,
                          joff, a.vt, a.tj, e.body.sparse, stream, body_blended);
    if (rc) return rc;
    // head splice (EHM.py:72-75, :121-124)
    if (fuse)
        rc = lbs_skin_splice(B, Vh, Jh, e.flame.sparse, a.ws_h, Vb, e.head_index, e.r_eyelid, e.l_eyelid, eyelid,
                             hscale, a.hj, e.hj0, e.hj1, a.tj, Jb, e.bj0, e.bj1, a.vt, e.bad_index_flag, stream);
    else
        rc = gsr_splice_head(B, Vb, Vh, e.head_index, a.hv, e.r_eyelid, e.l_eyelid, eyelid, hscale, a.hj, Jh, e.hj0,
                             e.hj1, a.tj, Jb, e.bj0, e.bj1, a.vt, e.bad_index_flag, stream);
    if (rc) return rc;
    // body lbs_wobeta (EHM.py:134-137)
    return gsr_lbs_sp(B, Vb, Jb, 0, a.vt, (int64_t)Vb * 3, nullptr, nullptr, a.pose_b, 1, e.body.posedirs,
                      e.body.J_regressor, e.body.parents_host, e.body.lbs_weights_t, joff, out->vertices,
                      out->joints_transform, out->joints, out->ver_transform_mat, out->joint_transform_mat, nullptr,
                      a.ws_b, e.body.sparse, stream);
}

}  // extern "C"
