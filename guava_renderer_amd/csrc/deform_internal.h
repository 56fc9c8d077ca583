// deform_internal.h -- library-internal entry points of deform.hip for ehm.hip (not part of the C ABI).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/gsr_deform.h"

namespace gsr {
// One single-frame blend over the tiled bases (k_lbs_blend_tiled1's arguments, deform.hip)
struct Blend1Job {
    int M, NB, NP, pose2rot;
    const float* vt;
    const float* betas;
    const float4* sd_tiled;
    const float* feat;
    const float4* pd_tiled;
    float* v_shaped;
    float* v_posed;
    const float* pose;
};
// whether launch_blend takes k_lbs_blend_tiled1 for these arguments, and that launch's job
bool blend_tiled1_applies(int B, int NB, int NP, const float* vp, const GsrLbsSparse* sp);
Blend1Job blend1_job(int M, int NB, int NP, const float* vt, const float* betas, const float* feat, float* vs,
                     float* vp, const GsrLbsSparse* sp, const float* pose, int pose2rot);
// gsr_blend_joints_sp; blend_done: its blend was launched already (as lbs_run's companion)
int blend_joints_run(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
                     const float* betas, const float* shapedirs_t, const float* J_regressor,
                     const float* joints_offset, float* v_shaped, float* joints, const GsrLbsSparse* sp,
                     void* stream, bool blend_done);
// gsr_lbs_sp; with skin = false it stops after the kinematic chain, leaving the joint transforms and
// v_posed in the workspace for lbs_skin_splice
int lbs_run(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride, const float* betas,
            const float* shapedirs_t, const float* pose, int pose2rot, const float* posedirs,
            const float* J_regressor, const int32_t* parents_host, const float* lbs_weights_t,
            const float* joints_offset, float* verts, float* joints_transformed, float* joints,
            float* vert_transforms, float* joint_transforms, float* v_shaped, char* workspace,
            const GsrLbsSparse* sp, void* stream, bool skin, const Blend1Job* companion = nullptr,
            bool* companion_done = nullptr);
// (companion: a single-frame blend independent of this call's, launched together with this call's
// blend when both take k_lbs_blend_tiled1; *companion_done says whether it was)
// the head's ELL skinning fused into gsr_splice_head's arithmetic (one launch); 1 = not applicable
// (no ELL weights: the caller skins and splices separately), 0 = launched, < 0 = error
int lbs_skin_splice(int B, int Vh, int Jh, const GsrLbsSparse* sp_h, const char* ws_h, int Vb,
                    const int32_t* head_index, const float* r_eyelid, const float* l_eyelid, const float* eyelid,
                    const float* head_scale, const float* head_joints, int hj0, int hj1, const float* body_joints,
                    int Jb, int bj0, int bj1, float* body_v_shaped, uint32_t* bad_index_flag, void* stream);
}  // namespace gsr
