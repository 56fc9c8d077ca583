/*
 * gsr_deform.h -- C ABI of the MI355X (gfx950) per-frame avatar deformation that feeds the
 * rasterizer.
 *
 * Each entry point replaces one function of the reference's torch code
 * (/root/reference/models/...):
 *
 *   gsr_lbs              <- lbs()                      modules/flame/lbs.py:142-229 (betas != NULL)
 *                           lbs_wobeta()               modules/flame/lbs.py:255-333 (betas == NULL)
 *                           with blend_shapes :355-376, vertices2joints :335-352,
 *                           batch_rodrigues :379-410, batch_rigid_transform :426-482 fused in.
 *                           Used by EHM.forward (modules/ehm/EHM.py:67-70 FLAME head,
 *                           :134-137 SMPL-X body).
 *   gsr_blend_joints     <- blend_shapes + vertices2joints (lbs.py:355-376, :335-352), the body
 *                           template step of EHM.forward (EHM.py:114-118)
 *   gsr_splice_head      <- EHM.forward's FLAME-head splice (EHM.py:72-75, :121-124)
 *   gsr_pack_rows        <- the torch.cat coefficient-row glue of EHM.forward (EHM.py:41-48, :94-112)
 *   gsr_deform_gaussians <- the Gaussian part of Ubody_Gaussian.forward
 *                           UbodyAvatar/ubody_gaussian.py:252-278: vertex Gaussians
 *                           (rotmat_to_unitquat of the per-vertex skinning matrix, quat_product,
 *                           normalize) and UV Gaussians (compute_face_orientation,
 *                           utils/graphics_utils.py:61-80, face binding, barycentric centre,
 *                           face-scaled local offset and scale), concatenated vertex-first.
 *
 * Conventions: device pointers, float32, the reference's layouts unless stated.  Two operands are
 * taken k-major (transposed once at avatar load, so the per-frame kernels read them coalesced):
 *   shapedirs_t   [NB, V*3]  = the reference's shapedirs [V,3,NB] permuted to (NB, V, 3)
 *   lbs_weights_t [J, V]     = the reference's lbs_weights [V,J] transposed
 * posedirs keeps the reference layout [(J-1)*9, V*3] (already k-major).  `parents` is a HOST array
 * of J int32 with parents[0] = -1 and 0 <= parents[i] < i (the order batch_rigid_transform walks).
 * Per-frame tensors with a `_stride` argument are [B, n, k] when the stride is n*k and shared by
 * every frame ([n, k]) when it is 0.  Return codes: 0 = success, < 0 = -gsr_status
 * (gsr_last_error() explains).
 */
#ifndef GSR_DEFORM_H
#define GSR_DEFORM_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_LBS_MAX_JOINTS 64

/* Scratch bytes for gsr_lbs (rotation matrices, pose features, v_shaped, v_posed, rest joints,
 * joint transforms of B frames). */
size_t gsr_lbs_workspace_bytes(int B, int V, int J, int NB);

/* lbs / lbs_wobeta for B frames.
 *   v_template [V,3] (stride 0) or [B,V,3] (stride V*3); for lbs_wobeta this is v_shaped.
 *   betas [B,NB] + shapedirs_t [NB,V*3], or betas == NULL (NB ignored): lbs_wobeta.
 *   pose: pose2rot != 0 -> [B,J,3] axis-angle (batch_rodrigues); 0 -> [B,J,9] rotation matrices.
 *   joints_offset [B,J,3] or NULL (added to the regressed joints, lbs.py:191/:295).
 * Outputs (each may be NULL except verts):
 *   verts [B,V,3]; joints_transformed [B,J,3] (posed joints); joints [B,J,3] (rest joints incl.
 *   offset, lbs_wobeta's J); vert_transforms [B,V,16] (row-major 4x4, EHM's ver_transform_mat);
 *   joint_transforms [B,J,16] (A, joint_transform_mat); v_shaped [B,V,3]. */
int gsr_lbs(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
            const float* betas, const float* shapedirs_t, const float* pose, int pose2rot,
            const float* posedirs, const float* J_regressor, const int32_t* parents_host,
            const float* lbs_weights_t, const float* joints_offset, float* verts,
            float* joints_transformed, float* joints, float* vert_transforms,
            float* joint_transforms, float* v_shaped, char* workspace, void* stream);

/* Sparse forms of two dense LBS assets, built once per avatar by the caller (EHMDeformer does it at
 * load).  Real SMPL-X / FLAME assets are sparse: a joint regresses a few dozen vertices and a vertex
 * is skinned by a few joints.  With them, gsr_lbs_sp / gsr_blend_joints_sp take one load round per
 * frame for the joints instead of a pass over J x V weights, and K (not J) weights per vertex.
 *   jreg_row [J+1], jreg_col [nnz] (vertex, increasing in a row), jreg_val [nnz]: J_regressor's
 *   nonzeros as CSR rows (NULL jreg_row: the dense J_regressor).  The joint sums are
 *   re-associated (per-lane chains + a fixed tree), deterministic run to run.
 *   skin_k in [1, 16] (0: the dense lbs_weights_t), skin_joint / skin_weight [skin_k, V]: per vertex
 *   its nonzero (joint, weight) pairs in increasing joint order, padded with weight 0 -- the dense
 *   skinning's fmaf chains minus their zero terms, so the vertices and transforms are identical.
 *   skin_joint values must be in [0, J) (the kernel clamps them to J-1, so a bad value gives a wrong
 *   vertex, never an out-of-range read).
 *   shapedirs_tiled / posedirs_tiled (or NULL): the blend-shape bases shapedirs_t [NB][3V] and
 *   posedirs [9(J-1)][3V] re-laid as 1-KB tiles of 32 coordinates x 8 k for 16-byte loads:
 *   float4 (t * ceil(K/8) + g) * 64 + 32 h + c, component j = base[8g + 4h + j][32t + c], zero-padded
 *   to K multiple of 8 and 3V multiple of 32 (gsr_lbs_tile_bases).  Used for B = 1 and B > 16; the
 *   k sums are re-associated (fixed order, deterministic).  *_tiled_k / *_tiled_m: the K and M the
 *   base was tiled for; a call whose NB (shape) or 9(J-1) (pose) and 3V differ is refused
 *   (GSR_ERR_ARG), since the tile indexing depends on both. */
typedef struct {
    const int32_t* jreg_row;
    const int32_t* jreg_col;
    const float* jreg_val;
    int32_t skin_k;
    int32_t pad_;
    const int32_t* skin_joint;
    const float* skin_weight;
    const float* shapedirs_tiled;
    const float* posedirs_tiled;
    int32_t shapedirs_tiled_k, shapedirs_tiled_m;
    int32_t posedirs_tiled_k, posedirs_tiled_m;
} GsrLbsSparse;
/* Floats of a tiled base (GsrLbsSparse.*_tiled) for K x M, and the re-layout of a k-major base
 * [K][M] (device pointers) into it. */
size_t gsr_lbs_tiled_floats(int K, int M);
int gsr_lbs_tile_bases(int K, int M, const float* base, float* tiled, void* stream);
#define GSR_LBS_SKIN_MAX_K 16

/* gsr_lbs with the sparse assets (sp may be NULL: gsr_lbs). */
int gsr_lbs_sp(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
               const float* betas, const float* shapedirs_t, const float* pose, int pose2rot,
               const float* posedirs, const float* J_regressor, const int32_t* parents_host,
               const float* lbs_weights_t, const float* joints_offset, float* verts,
               float* joints_transformed, float* joints, float* vert_transforms,
               float* joint_transforms, float* v_shaped, char* workspace, const GsrLbsSparse* sp,
               void* stream);

/* blend_shapes + vertices2joints (lbs.py:355-376, :335-352; EHM.py:115-118): v_shaped [B,V,3] =
 * v_template + shapedirs . betas (betas == NULL: a copy of v_template), joints [B,J,3] =
 * J_regressor . v_shaped (+ joints_offset [B,J,3] or NULL). */
int gsr_blend_joints(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
                     const float* betas, const float* shapedirs_t, const float* J_regressor,
                     const float* joints_offset, float* v_shaped, float* joints, void* stream);
/* gsr_blend_joints with the sparse J_regressor (sp may be NULL). */
int gsr_blend_joints_sp(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
                        const float* betas, const float* shapedirs_t, const float* J_regressor,
                        const float* joints_offset, float* v_shaped, float* joints, const GsrLbsSparse* sp,
                        void* stream);

/* EHM.forward's head splice (EHM.py:72-75, :121-124) into the body template, in place:
 *   h = (head_verts + r_eyelid * eyelid[:,1] + l_eyelid * eyelid[:,0]) * head_scale
 *   body_v_shaped[b, head_index[i]] = h - mean(head_joints[b, hj0:hj1]) + mean(body_joints[b, bj0:bj1])
 * head_verts [B,N_head,3] (FLAME lbs output), r/l_eyelid [N_head,3], eyelid_params [B,2] (or NULL:
 * no eyelids), head_scale [B,3] (or NULL), head_joints [B,J_head,3], body_joints [B,J_body,3]
 * (EHM: hj = [3,5), bj = [23,25)).  An out-of-range head_index ORs 2 into *bad_index_flag. */
int gsr_splice_head(int B, int V_body, int N_head, const int32_t* head_index, const float* head_verts,
                    const float* r_eyelid, const float* l_eyelid, const float* eyelid_params,
                    const float* head_scale, const float* head_joints, int J_head, int hj0, int hj1,
                    const float* body_joints, int J_body, int bj0, int bj1, float* body_v_shaped,
                    uint32_t* bad_index_flag, void* stream);

/* The avatar pipeline's fused forward (round 4): gsr_forward_batch for the Gaussians of
 * gsr_deform_gaussians WITHOUT materialising them -- one kernel assembles each (Gaussian, frame)'s
 * mean, rotation and scale from the deformed mesh (ubody_gaussian.py:252-278) and projects it
 * (forward.cu:151-269) from registers, so the 40 B per Gaussian-frame the assembly would write and
 * preprocess would read never reach HBM.  P = V + N Gaussians, vertex ones first; colors / opacities
 * [P,k] (stride 0) or [B,P,k] as in gsr_forward_batch.  Images identical to gsr_deform_gaussians +
 * gsr_forward_batch (same kernels' arithmetic).  Forward-only (GSR_FORWARD_ONLY is implied: no backward
 * can use the workspace, the deformed attributes are not kept). */
typedef struct {
    int V, F, N, pad_;
    const float* verts;            /* [B,V,3] deformed mesh (EHM vertices) */
    const float* vert_transforms;  /* [B,V,4,4] */
    const int32_t* faces;          /* [F,3] */
    const float* vtx_rotations; int64_t vtx_rot_stride;   /* [V,4] wxyz (stride 0) or per frame */
    const float* vtx_scales; int64_t vtx_scale_stride;
    const int32_t* binding_face;   /* [N] */
    const float* face_bary;        /* [N,3] */
    const float* local_xyz; int64_t local_stride;
    const float* uv_rotations; int64_t uv_rot_stride;
    const float* uv_scales; int64_t uv_scale_stride;
    uint32_t* bad_index_flag;      /* ORed with 1 on an out-of-range binding (those Gaussians NaN) */
} GsrDeformInputs;
int gsr_forward_batch_deformed(int B, int width, int height, const GsrDeformInputs* dg, const float* colors,
                               int64_t colors_stride, const float* opacities, int64_t opac_stride,
                               float scale_modifier, const float* viewmatrices, const float* projmatrices,
                               const float* tanfov, const float* backgrounds, int64_t bg_stride,
                               char* workspace, int64_t R_capacity, float* out_color, float* out_invdepth,
                               int* radii, int antialiasing, uint32_t numerics, void* stream);

/* One segment of gsr_pack_rows: for every frame b, dst[b * dst_stride + c] = src[b * src_stride + c]
 * for c in [0, width) (src == NULL writes zeros; src_stride 0 broadcasts one row to every frame). */
typedef struct {
    const float* src;
    float* dst;
    int64_t src_stride;
    int64_t dst_stride;
    int32_t width;
    int32_t pad_;
} GsrRowSegment;
#define GSR_PACK_MAX_SEGMENTS 16

/* Assembles per-frame coefficient rows from pieces in ONE launch: the torch.cat / zeros / expand
 * glue of EHM.forward (EHM.py:41-48 FLAME betas and pose, :94-112 SMPL-X shape ++ expression and
 * the 55-joint pose with zero jaw/eyes, head_scale's broadcast).  nseg <= GSR_PACK_MAX_SEGMENTS,
 * width <= 4096; segments must not overlap. */
int gsr_pack_rows(int B, int nseg, const GsrRowSegment* segs, void* stream);

/* EHM.forward (modules/ehm/EHM.py:36-156) for B frames in ONE host call: the coefficient-row glue
 * (:41-48, :94-112, one pack launch), the FLAME head lbs (:67-70), the body template's blend shapes
 * and joints (:114-118), the head splice with eyelids and head scale (:72-75, :121-124) and the body
 * lbs_wobeta (:134-137) -- the same kernels as gsr_pack_rows + gsr_lbs_sp + gsr_blend_joints_sp +
 * gsr_splice_head + gsr_lbs_sp, issued from C so a single-frame call pays one FFI crossing instead of
 * five plus the host-side table building (the per-frame drop-in loop is host-bound there).
 *
 * One LBS model (GsrEhmModel): the assets of gsr_lbs_sp in its layouts; NB = the blend's shape
 * coefficients (FLAME: shape + expression (+ zero padding); SMPL-X: shape + expression). */
typedef struct {
    int32_t V, J, NB, pad_;
    const float* v_template;      /* [V,3] */
    const float* shapedirs_t;     /* [NB, 3V] */
    const float* posedirs;        /* [9(J-1), 3V] */
    const float* J_regressor;     /* [J, V] */
    const float* lbs_weights_t;   /* [J, V] */
    const int32_t* parents_host;  /* HOST [J] */
    const GsrLbsSparse* sparse;   /* or NULL */
} GsrEhmModel;
typedef struct {
    GsrEhmModel flame, body;
    const int32_t* head_index;    /* [N_head] smplx2flame_ind: body vertex of each FLAME vertex */
    const float* l_eyelid;        /* [N_head,3] */
    const float* r_eyelid;        /* [N_head,3] */
    int32_t N_head;               /* = flame.V */
    int32_t hj0, hj1, bj0, bj1;   /* splice reference joints (EHM: head [3,5), body [23,25)) */
    int32_t pad_;
    uint32_t* bad_index_flag;     /* device, ORed with 2 on an out-of-range head_index (or NULL) */
} GsrEhm;
/* One per-frame parameter: rows of `width` floats, row b at p + b * row_stride (row_stride 0: one
 * row for every frame); p == NULL: absent (its columns stay zero, as the reference's zeros). */
typedef struct {
    const float* p;
    int64_t row_stride;
    int32_t width, pad_;
} GsrEhmParam;
/* The parameters' slots in the `params` array (the reference's dict keys):
 * flame_param_dict shape_params, expression_params, jaw_params, eye_pose_params, eyelid_params;
 * body_param_dict shape, exp, global_pose, body_pose, left_hand_pose, right_hand_pose, head_scale,
 * joints_offset. */
enum {
    GSR_EHM_FLAME_SHAPE = 0, GSR_EHM_FLAME_EXPR, GSR_EHM_FLAME_JAW, GSR_EHM_FLAME_EYES, GSR_EHM_FLAME_EYELID,
    GSR_EHM_BODY_SHAPE, GSR_EHM_BODY_EXP, GSR_EHM_BODY_GLOBAL, GSR_EHM_BODY_POSE, GSR_EHM_BODY_LHAND,
    GSR_EHM_BODY_RHAND, GSR_EHM_BODY_HEAD_SCALE, GSR_EHM_BODY_JOINTS_OFFSET, GSR_EHM_NPARAM
};
/* EHM.forward's output dict; every pointer but vertices may be NULL. */
typedef struct {
    float* vertices;              /* [B,Vb,3] */
    float* joints;                /* [B,Jb,3] rest joints incl. offset */
    float* joints_transform;      /* [B,Jb,3] posed joints */
    float* ver_transform_mat;     /* [B,Vb,16] */
    float* joint_transform_mat;   /* [B,Jb,16] */
} GsrEhmOutputs;
/* Scratch bytes of gsr_ehm_forward for B frames (coefficient rows, the head's vertices and joints,
 * the body template and joints, and both lbs workspaces). */
size_t gsr_ehm_workspace_bytes(const GsrEhm* ehm, int B);
/* Column layout (EHM.py): FLAME betas = shape ++ expression ++ zeros (flame.NB wide); FLAME pose =
 * 0 global, 0 neck, jaw at column 6, eyes at 9 (3 * flame.J wide); body betas = shape (cut to
 * body.NB - exp width, as the reference slices it) ++ zeros ++ exp at body.NB - exp width; body pose
 * = global_pose (its first 3 columns) at 0, body_pose (first 63) at 3, zero jaw and eyes, left hand
 * at 75, right hand at 120 (3 * body.J wide).  eyelid_params must be 2 wide, head_scale 3,
 * joints_offset 3 * body.J.  A parameter that does not fit its columns is refused (GSR_ERR_ARG)
 * before any launch. */
int gsr_ehm_forward(const GsrEhm* ehm, int B, const GsrEhmParam* params, const GsrEhmOutputs* out,
                    char* workspace, void* stream);

/* Ubody_Gaussian.forward's Gaussian assembly for B frames; P = V + N Gaussians per frame, the V
 * vertex Gaussians first.
 *   verts [B,V,3], vert_transforms [B,V,16] (from gsr_lbs), faces [F,3] int32.
 *   vertex Gaussians: rotations [V,4] wxyz and scales [V,3] (with strides: shared or per frame).
 *   UV Gaussians: binding_face [N] int32 in [0,F), face_bary [N,3], local_xyz [N,3],
 *   rotations [N,4] wxyz, scales [N,3] (local/rot/scale with strides).
 * Outputs: means3D [B,P,3], rotations [B,P,4] wxyz, scales [B,P,3].  Indices are validated on the
 * device: an out-of-range binding face or face-vertex index ORs 1 into *bad_index_flag (a device
 * uint32, may be NULL) and writes NaN for that Gaussian instead of reading out of range (the
 * reference raises IndexError).  compute_face_orientation runs once per (face, frame) as in the
 * reference when a 256-Gaussian block's bindings span at most 256 consecutive faces (GUAVA's texel
 * order), else once per bound Gaussian; the results are the same. */
int gsr_deform_gaussians(int B, int V, int F, int N, const float* verts,
                         const float* vert_transforms, const int32_t* faces,
                         const float* vtx_rotations, int64_t vtx_rot_stride,
                         const float* vtx_scales, int64_t vtx_scale_stride,
                         const int32_t* binding_face, const float* face_bary,
                         const float* local_xyz, int64_t local_stride,
                         const float* uv_rotations, int64_t uv_rot_stride,
                         const float* uv_scales, int64_t uv_scale_stride, float* means3D,
                         float* rotations, float* scales, uint32_t* bad_index_flag, void* stream);

#ifdef __cplusplus
}
#endif
#endif
