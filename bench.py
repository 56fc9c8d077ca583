#!/usr/bin/env python
"""Headline benchmark: rendered frames/sec at 512x512 with ~100k Gaussians (BASELINE.json).

One step = one pass of GUAVA's per-frame animation path over a batch of `--batch` tracked frames
(config 2 "self-reenactment": main/test.py:70-76 times Ubody_Gaussian.forward + render per frame):
  --pipeline avatar (default): EHM deformation (FLAME head LBS + SMPL-X body LBS, per-frame pose,
      expression, eyelids), vertex + UV Gaussian assembly, then the rasterizer hot path
      (preprocess -> tile binning -> per-tile depth order -> 32-channel compositing);
  --pipeline raster: the rasterizer alone over one static cloud seen by a camera per frame.
Synthetic avatar: P=100,000 Gaussians (10,475 SMPL-X vertex Gaussians + UV Gaussians), 512x512,
one camera and one pose per frame; every input resident in HBM before the timed region.  N GPUs: one process per GPU, each renders its
own `--batch` frames (frames are independent -> weak scaling, no collective in the data path;
torch.distributed is used only for the barrier and the max-over-ranks time).

Prints ONE JSON line (rank 0) with the contract fields plus:
  roofline      -- render_fwd kernel: algorithmic bytes per launch / average launch time from HIP
                   events recorded on the launch stream inside the timed region;
  cpu_baseline  -- the CPU oracle (a port of the reference algorithm) timed on a bounded sample of
                   the same workload on this host's cores (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TFLOPS = 157.3  # dense f32-input MFMA peak (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak (MI355X_MICROARCH.md, no sparsity)
C = 32


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32, help="frames per step per GPU")
    ap.add_argument("--config", default="c2", choices=["c2", "c5"])
    ap.add_argument("--pipeline", default="avatar", choices=["avatar", "raster", "train", "frame"],
                    help="train = BASELINE config 4: raster fwd + fused-SSIM/L1 loss + raster bwd + "
                         "gradient all-reduce + Adam (use --batch 6); frame = GUAVA's unchanged caller: "
                         "one GaussianRasterizer_32 call per frame as gaussian_render.py:37-67 does")
    ap.add_argument("--inflight", type=int, default=1,
                    help="batches in flight on separate HIP streams (avatar/raster pipelines): the deform "
                         "and binning of one batch overlap the compositing of the others (3: +4%% frames/s "
                         "over 1); kernel times for the roofline then come from an isolated pass")
    ap.add_argument("--refine", action="store_true",
                    help="fuse the refiner's first 1x1 conv 32->16 + leaky ReLU into the render "
                         "epilogue (inference output: 16 refiner features + 4 raw channels)")
    ap.add_argument("--fast-exp", action="store_true", help="hardware exp (not bit-exact)")
    ap.add_argument("--exact-accum", action="store_true",
                    help="f32 MFMA colour accumulation, bit-identical to the oracle (default: split-bf16 "
                         "MFMA accumulation, colour within the north_star's 1e-4 L_inf, include/gsr.h)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stages", action="store_true", help="also time every stage (extra events)")
    return ap.parse_args()


def _workload(cfg):
    if cfg == "c5":
        return dict(P=300000, W=1024, H=1024, gpt=3, name="guava-avatar-synth-300k-1024")
    return dict(P=100000, W=512, H=512, gpt=1, name="guava-avatar-synth-100k-512")


def _render_alg_bytes(P_vis, W, H):
    # render_fwd compulsory traffic per frame: per visible Gaussian its 32 features (128 B) +
    # means2D (8) + conic/opacity (16) + 1/depth (4); per pixel 32 channels + inverse depth out
    # (132 B) + final_T + n_contrib (8 B) kept for backward.
    return 156.0 * P_vis + 140.0 * W * H


def _render_bwd_alg_bytes(P_vis, W, H):
    # render_bwd compulsory traffic per frame: per pixel dL/dpixel (32 channels) + dL/dinvdepth read
    # (132 B) + final_T + n_contrib (8 B); per visible Gaussian its render record (32 B) and 32
    # features (128 B) read, its colour gradient (128 B) and 7 screen-space terms (28 B) written.
    return 316.0 * P_vis + 140.0 * W * H


def _path_alg_bytes(P, W, H):
    # SURVEY.md 8(d) / BASELINE.md: B_fwd = 176*P + 132*H*W per frame
    return 176.0 * P + 132.0 * W * H


def cpu_baseline(scene, cams, W, H, budget_s, avatar_inputs=None):
    """The CPU oracle timed on a bounded sample of the same workload (rank 0, N=1)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # CPU restatement of the reference algorithm (checker / baseline only)
    import lbs_oracle  # CPU restatement of the deformation (numpy)
    # the cores this process may use (affinity), capped by OMP_NUM_THREADS where the host sets it
    # (the GPU box: 16 per GPU job)
    threads = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        threads = min(threads, int(omp))
    oracle.set_threads(threads)
    bg = np.zeros(C, np.float32)
    t0 = time.perf_counter()
    frames = 0
    while True:
        i = frames % len(cams)
        cam = cams[i]
        means, rots, scales = scene.get("means3D"), scene.get("rotations"), scene.get("scales")
        if avatar_inputs is not None:  # deform this frame on the CPU too
            body, flame, extra, g, bp, fp = avatar_inputs
            one = lambda d: {k: v[i:i + 1] for k, v in d.items()}  # noqa: E731
            e = lbs_oracle.ehm_forward(body, flame, extra, one(bp), one(fp))
            dg = lbs_oracle.deform_gaussians(e["vertices"], e["ver_transform_mat"], extra["faces"],
                                             g["vtx_rotations"], g["vtx_scales"], g["binding_face"],
                                             g["face_bary"], g["local_xyz"], g["uv_rotations"],
                                             g["uv_scales"])
            means = dg["xyz"][0].astype(np.float32)
            rots = dg["rotation"][0].astype(np.float32)
            scales = dg["scaling"][0].astype(np.float32)
        oracle.forward(means, scene["colors"], scene["opacities"], scales, rots, None,
                       cam["viewmatrix"], cam["projmatrix"], W, H, cam["tanfovx"], cam["tanfovy"], bg)
        frames += 1
        el = time.perf_counter() - t0
        if el >= budget_s or frames >= 512:
            break
    model = "unknown CPU"
    try:
        model = next(ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    what = "deform (numpy) + preprocess+bin+sort+render (C)" if avatar_inputs is not None else \
        "preprocess+bin+sort+render"
    return dict(value=frames / el, unit="frames/s", cores=threads, kind="port",
                sample=f"{frames} frames of the same {W}x{H} workload through the CPU oracle "
                       f"({what}, OpenMP {threads} threads on {model}) in {el:.1f}s")


def main():
    a = _args()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one process per GPU (RCCL = the "nccl" backend).  GSR_DIST_BACKEND=gloo rehearses the N>1
    # path with several ranks on one GPU (device = LOCAL_RANK modulo the visible devices).
    backend = os.environ.get("GSR_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(dev)

    from guava_renderer_amd import _lib, parallel, scenes
    from guava_renderer_amd.batch import BatchRasterizer, profile_enable, profile_read, render_counters
    _lib.set_exact_exp(not a.fast_exp)
    _lib.set_split_bf16(not a.exact_accum)

    wl = _workload(a.config)
    P, W, H, B = wl["P"], wl["W"], wl["H"], a.batch
    cams_all = scenes.frame_cameras(B * world, W, H, seed=1000)
    cams = parallel.shard_frames(cams_all, rank, world)  # B frames per rank, no data-path collective
    t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
    views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
    projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
    tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
    bgs = torch.zeros((B, C), dtype=torch.float32, device=dev)
    avatar_inputs = None
    workload = wl["name"] + {"avatar": "-deform+raster", "raster": "-raster", "train": "-train",
                             "frame": "-per-frame-dropin"}[a.pipeline]

    if a.pipeline == "avatar":
        from guava_renderer_amd import avatar
        from guava_renderer_amd.pipeline import AvatarPipeline
        body, flame, extra = avatar.ehm_assets(seed=0)
        verts, faces, tex = avatar.template_mesh()
        g = avatar.gaussians(verts, faces, tex, P=P, seed=0)
        bp_all, fp_all = avatar.ehm_params(B * world, seed=1000)
        lo, hi = parallel.shard_range(B * world, rank, world)
        bp = {k: v[lo:hi] for k, v in bp_all.items()}
        fp = {k: v[lo:hi] for k, v in fp_all.items()}
        bpt = {k: t(v) for k, v in bp.items()}
        fpt = {k: t(v) for k, v in fp.items()}
        probe = AvatarPipeline(body, flame, extra, g, B, W, H, R_capacity=24 * P * B, device=dev)
        probe.render(bpt, fpt, views, projs, tanf)
        R_probe, ovf = probe.rast.status()
        assert not ovf, "probe overflow"
        del probe
        torch.cuda.empty_cache()
        pipes = [AvatarPipeline(body, flame, extra, g, B, W, H, R_capacity=int(R_probe * 1.25) + 1024, device=dev)
                 for _ in range(max(1, a.inflight))]
        pipe = pipes[0]
        P = pipe.P
        rast = pipe.rast
        rasts = [p.rast for p in pipes]
        scene = {"colors": g["colors"], "opacities": g["opacities"]}
        avatar_inputs = (body, flame, extra, g, bp, fp)

        head = None
        if a.refine:
            from guava_renderer_amd.batch import RefineHead
            rng = np.random.default_rng(5)  # random-init conv_body_first (nn.Conv2d(32, 16, 1))
            head = RefineHead(t(rng.uniform(-0.18, 0.18, (16, 32)).astype(np.float32)),
                              t(rng.uniform(-0.18, 0.18, 16).astype(np.float32)), keep_channels=4)

        def step_on(i):
            return pipes[i].render(bpt, fpt, views, projs, tanf, refine=head)
    elif a.pipeline == "train":
        from guava_renderer_amd.train import SplatTrainer
        scene = scenes.avatar_cloud(P, seed=0, gaussians_per_texel=wl["gpt"])
        P = scene["means3D"].shape[0]
        params = {k: t(scene[k]) for k in ("means3D", "colors", "opacities", "scales", "rotations")}
        probe = BatchRasterizer(B, P, W, H, R_capacity=24 * P * B, device=dev)
        probe.forward(params["means3D"], params["colors"], params["opacities"], params["scales"],
                      params["rotations"], views, projs, tanf, bgs)
        R_probe, ovf = probe.status()
        assert not ovf, "probe overflow"
        del probe
        torch.cuda.empty_cache()
        # the trainable parameters are the raw attributes: a small learning rate
        # keeps the per-step work at the avatar's distribution over the timed steps; capacity with
        # headroom for the drift (an overflowing step is skipped on the device and counted)
        trainer = SplatTrainer(params, B, W, H, R_capacity=int(R_probe * 2) + 1024, device=dev, lr=1e-5)
        rast = trainer.rast
        target = torch.rand((B, 3, H, W), device=dev, generator=torch.Generator(device=dev).manual_seed(rank))

        rasts = [rast]

        def step_on(i):
            return trainer.step(views, projs, tanf, target)
    elif a.pipeline == "frame":
        # GUAVA's unchanged caller (models/UbodyAvatar/gaussian_render.py:19-67, the refiner aside):
        # one GaussianRasterizationSettings + GaussianRasterizer_32 call per frame, camera fields
        # read per frame with int()/float() from device tensors, outputs stacked.  The deformed
        # assets of the B frames come from the deform kernels, outside the timed region.
        from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32
        from guava_renderer_amd import avatar
        from guava_renderer_amd.pipeline import AvatarPipeline
        body, flame, extra = avatar.ehm_assets(seed=0)
        verts, faces, tex = avatar.template_mesh()
        g = avatar.gaussians(verts, faces, tex, P=P, seed=0)
        bp_all, fp_all = avatar.ehm_params(B * world, seed=1000)
        lo, hi = parallel.shard_range(B * world, rank, world)
        bpt = {k: t(v[lo:hi]) for k, v in bp_all.items()}
        fpt = {k: t(v[lo:hi]) for k, v in fp_all.items()}
        dpipe = AvatarPipeline(body, flame, extra, g, B, W, H, R_capacity=24 * P * B, device=dev)
        dg = dpipe.deform(bpt, fpt)
        P = dpipe.P
        assets = {"xyz": dg["xyz"], "rotation": dg["rotation"], "scaling": dg["scaling"],
                  "opacity": dpipe.gauss.opacity.unsqueeze(0).expand(B, -1, -1),
                  "features_color": dpipe.gauss.colors.unsqueeze(0).expand(B, -1, -1)}
        cam_params = {"image_height": torch.full((B,), H, device=dev), "image_width": torch.full((B,), W, device=dev),
                      "tanfovx": tanf[:, 0].contiguous(), "tanfovy": tanf[:, 1].contiguous(),
                      "world_view_transform": views.view(B, 4, 4), "full_proj_transform": projs.view(B, 4, 4),
                      "camera_center": t(np.stack([c["campos"] for c in cams]))}
        scene = {"colors": g["colors"], "opacities": g["opacities"]}
        avatar_inputs = (body, flame, extra, g, {k: v[lo:hi] for k, v in bp_all.items()},
                         {k: v[lo:hi] for k, v in fp_all.items()})
        rasts = []
        last_radii = [None]

        def step_on(i):
            with torch.no_grad():
                mean_3d = assets["xyz"]
                features_color = assets["features_color"].clone()
                mean_2d = torch.zeros_like(mean_3d, dtype=torch.float32, requires_grad=True, device=dev)
                bg = torch.ones((B, features_color.shape[-1]), dtype=torch.float32, device=dev) * 0.0
                imgs, radiis, depths = [], [], []
                for bi in range(B):
                    rs = GaussianRasterizationSettings(
                        image_height=int(cam_params["image_height"][bi]), image_width=int(cam_params["image_width"][bi]),
                        tanfovx=float(cam_params["tanfovx"][bi]), tanfovy=float(cam_params["tanfovy"][bi]),
                        bg=bg[bi], scale_modifier=1.0, viewmatrix=cam_params["world_view_transform"][bi],
                        projmatrix=cam_params["full_proj_transform"][bi], sh_degree=0,
                        campos=cam_params["camera_center"][bi], prefiltered=False, debug=False, antialiasing=False)
                    img, rad, dep = GaussianRasterizer_32(raster_settings=rs)(
                        means3D=mean_3d[bi], means2D=mean_2d[bi], shs=None, colors_precomp=features_color[bi],
                        opacities=assets["opacity"][bi], scales=assets["scaling"][bi],
                        rotations=assets["rotation"][bi], cov3D_precomp=None)
                    imgs.append(img)
                    radiis.append(rad)
                    depths.append(dep)
                out = torch.stack(imgs, 0)
                last_radii[0] = torch.stack(radiis, 0)
                return out, torch.stack(depths, 0), last_radii[0]
    else:
        scene = scenes.avatar_cloud(P, seed=0, gaussians_per_texel=wl["gpt"])
        P = scene["means3D"].shape[0]
        means, colors = t(scene["means3D"]), t(scene["colors"])
        opac, scales, rots = t(scene["opacities"]), t(scene["scales"]), t(scene["rotations"])
        # size the instance capacity from one probe batch
        probe = BatchRasterizer(B, P, W, H, R_capacity=24 * P * B, device=dev)
        probe.forward(means, colors, opac, scales, rots, views, projs, tanf, bgs)
        R_probe, ovf = probe.status()
        assert not ovf, "probe overflow"
        del probe
        torch.cuda.empty_cache()
        rasts = [BatchRasterizer(B, P, W, H, R_capacity=int(R_probe * 1.25) + 1024, device=dev)
                 for _ in range(max(1, a.inflight))]
        rast = rasts[0]

        def step_on(i):
            return rasts[i].forward(means, colors, opac, scales, rots, views, projs, tanf, bgs)

    # batches in flight: step k runs on stream k mod n with its own pipeline / workspace (each
    # batch is complete work -- deform, binning, compositing; only consecutive batches overlap)
    n_inflight = max(1, len(rasts))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(n_inflight - 1)]
    step_count = [0]

    gather = dist is not None and a.pipeline != "train"
    # consumer boundary: every rank receives all ranks' RGB frames (RCCL all-gather over xGMI),
    # each batch's exchange overlapped with the next batch's rendering on a side stream
    gatherer = None
    if gather:
        gdev = dev if backend == "nccl" else torch.device("cpu")
        gatherer = parallel.FrameGather(B, (3, H, W), torch.float32, gdev)

    def step():
        i = step_count[0] % n_inflight
        step_count[0] += 1
        with torch.cuda.stream(streams[i]):
            res = step_on(i)
            if gatherer is not None:
                rgb = res[0][:, :3]
                gatherer.push(rgb if backend == "nccl" else rgb.cpu())
            return res

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if rasts:
        R_total, ovf = rast.status()
        assert not any(r.status()[1] for r in rasts)
        P_vis = int((rast.radii > 0).sum().item())
    else:  # per-frame drop-in path: the _C calls size their own buffers (exact R, host sync)
        R_total = None
        P_vis = int((last_radii[0] > 0).sum().item())
    profile_read()  # reset accumulators
    stage_set = (("preprocess", "scan", "depth_sort", "chunk_count", "tile_scan", "ordered_scatter",
                  "render_fwd", "render_bwd", "preprocess_bwd") if a.stages else
                 ("render_fwd", "render_bwd") if a.pipeline == "train" else ("render_fwd",))
    # with batches overlapping, a kernel's event-timed duration includes the other batch's work:
    # the timed region then carries no stage events, and the kernel times (roofline) come from an
    # isolated pass afterwards, one batch at a time
    isolated = n_inflight > 1
    profile_enable(() if isolated else stage_set)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    if gatherer is not None:
        gatherer.wait()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    prof = profile_read()
    profile_enable(())
    if isolated:
        profile_enable(stage_set)
        for _ in range(max(20, a.steps // 4)):
            with torch.cuda.stream(streams[0]):
                step_on(0)
        torch.cuda.synchronize(dev)
        prof = profile_read()
        profile_enable(())
    deform_ms = None
    if a.pipeline == "avatar":  # deformation alone (EHM + Gaussian assembly), outside the timed region
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            pipe.deform(bpt, fpt)
        e1.record()
        torch.cuda.synchronize(dev)
        deform_ms = e0.elapsed_time(e1) / a.steps
    # the bit-exact colour accumulation on the same workload (split-bf16 off), a shorter run after
    # the timed region: the line's `exact_accum` (N=1 avatar / raster pipelines, default mode only)
    exact_line = None
    if dist is None and not a.exact_accum and a.pipeline in ("avatar", "raster"):
        _lib.set_split_bf16(False)
        n_ex = max(20, a.steps // 4)
        for _ in range(3):
            step()
        torch.cuda.synchronize(dev)
        t_ex = time.perf_counter()
        for _ in range(n_ex):
            step()
        torch.cuda.synchronize(dev)
        ms_ex = (time.perf_counter() - t_ex) / n_ex * 1e3
        _lib.set_split_bf16(True)
        exact_line = {"value": round(1e3 * B / ms_ex, 2), "ms_per_step": round(ms_ex, 4), "steps": n_ex,
                      "colour_accum": "f32 mfma (bit-exact with the oracle)"}
    # work counters of one extra (instrumented, untimed) step: which wall the render kernel hits
    work = render_counters(step, device=dev)
    if a.pipeline == "train":
        assert trainer.skipped_steps == 0 and not trainer.rast.status()[1], "capacity overflow inside the timed region"
    else:
        assert not any(r.status()[1] for r in rasts), "capacity overflow inside the timed region"
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())

    frames = world * B * a.steps
    fps = frames / el
    ms_step = 1000.0 * el / a.steps
    rms, rcnt = prof.get("render_fwd", (0.0, 0))
    render_ms = rms / max(rcnt, 1)
    frames_per_launch = 1 if a.pipeline == "frame" else B
    bytes_launch = _render_alg_bytes(P_vis / B, W, H) * frames_per_launch
    achieved = bytes_launch / (render_ms * 1e-3) / 1e9 if render_ms > 0 else None
    traffic = issue = None
    # HBM traffic per launch from the committed PMC summaries (tools/pmc_summary.py): the contract
    # workload's (pmc_render_fwd.json) and the training batch's (pmc_train.json: render_fwd and
    # render_bwd of `--pipeline train --batch 6`)
    pmc_path = os.path.join(ROOT, "profiles", "pmc_train.json" if a.pipeline == "train" else "pmc_render_fwd.json")
    bwd_traffic = None
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if pm.get("config") == workload and pm.get("batch") == B:
                traffic = pm.get("hbm_bytes_per_launch")
                issue = pm.get("render_fwd_issue")
                bwd_traffic = (pm.get("kernels", {}).get("k_render_bwd") or {}).get("hbm_bytes")
        except Exception:  # noqa: BLE001
            traffic = None

    out = {
        "metric": ("training frames/sec (raster fwd+bwd + fused-SSIM loss) @512x512, ~100k Gaussians"
                   if a.pipeline == "train" else
                   "rendered frames/sec @512x512, ~100k Gaussians" if a.config == "c2"
                   else "rendered frames/sec @1024x1024, ~300k Gaussians"),
        "value": round(fps, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if a.exact_accum else "f32 (colour products in split-bf16: f = f_hi + f_lo, f32 accumulation)",
        "data": ("synthetic avatar (SMPL-X template mesh + UV-texel Gaussians, synthetic LBS bases, "
                 "GUAVA attribute distributions), one pose + one orbit camera per frame"
                 if a.pipeline == "avatar" else
                 "synthetic (SMPL-X-template avatar cloud, GUAVA attribute distributions, "
                 "one orbit camera per frame)"),
        "config": {"workload": workload,
                   "pipeline": {"avatar": "EHM LBS -> Gaussian assembly -> rasterize",
                                "raster": "rasterize",
                                "train": "raster fwd -> L1 + fused SSIM (raw RGB) + L1 of a fixed 32->3 refine stand-in "
                                         "(all 32 channels carry gradient) -> frame-reduced raster bwd -> "
                                         "grad all-reduce -> Adam",
                                "frame": "deformed frames -> GaussianRasterizer_32 once per frame (gaussian_render.py:37-67)"
                                }[a.pipeline] + (" + fused refiner conv_body_first" if a.refine else ""), "gaussians": P, "image": [W, H], "channels": C,
                   "frames_per_step_per_gpu": B, "global_batch": B * world,
                   "parallelism": f"frame-sharded x{world}" + (", RGB all-gather per step (overlapped with the next step)" if world > 1 and a.pipeline != "train" else ""),
                   "batches_in_flight": n_inflight,
                   "exp": "hw" if a.fast_exp else "exact-poly",
                   "colour_accum": "f32 mfma (bit-exact)" if a.exact_accum else "split-bf16 mfma (<=1e-4)",
                   "instances_per_step": R_total, "visible_gaussians_per_frame": P_vis / B},
        "roofline": {"bound": "hbm", "kernel": "render_fwd",
                     "achieved": round(achieved, 1) if achieved else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "alg_bytes_per_launch": bytes_launch,
                     "avg_launch_ms": round(render_ms, 4),
                     "timing": "isolated pass, one batch in flight" if isolated else "timed region"},
        "path_roofline": {"alg_bytes_per_frame": _path_alg_bytes(P, W, H),
                          "achieved_GBs": round(_path_alg_bytes(P, W, H) * fps / 1e9, 1),
                          "frac": round(_path_alg_bytes(P, W, H) * fps / 1e9 / HBM_PEAK_GBS, 4)},
    }
    # per-frame work of the render kernel and its matrix-core utilisation (dense peak of the MFMA used)
    ksteps = work["mfma_ksteps"]
    if a.exact_accum:
        mfma_flops = ksteps * 2 * (2 * 32 * 32 * 2)  # two v_mfma_f32_32x32x2f32 per wave k-step
    else:  # two v_mfma_f32_32x32x8_bf16 per wave k-step (every k-slot carries a split product)
        mfma_flops = ksteps * 2 * (2 * 32 * 32 * 8)
    out["render_work_per_frame"] = {k: round(v / B, 1) for k, v in work.items()}
    out["render_mfma"] = {"issued_tflops": round(mfma_flops / (render_ms * 1e-3) / 1e12, 2) if render_ms else None,
                          "peak_tflops": F32_MFMA_PEAK_TFLOPS if a.exact_accum else BF16_MFMA_PEAK_TFLOPS,
                          "instruction": "v_mfma_f32_32x32x2_f32" if a.exact_accum else "v_mfma_f32_32x32x8_bf16",
                          "useful_frac": round(work["pairs_contributing"] / max(64 * work["strip_pairs_blended"], 1), 4)}
    if issue is not None and not a.exact_accum:
        # the compute wall beside the HBM one: per-launch instruction counts and per-SIMD pipe busy
        # of the contract kernel, from the committed PMC passes (profiles/pmc_render_fwd.json)
        out["render_issue"] = dict(issue, source="profiles/pmc_render_fwd.json (tools/gpu_pmc_fwd.sh)",
                                   valu_per_kstep=round(issue["valu_insts"] / max(ksteps, 1), 1)
                                   if issue.get("valu_insts") else None)
    if a.pipeline == "train":
        bms, bcnt = prof.get("render_bwd", (0.0, 0))
        bwd_ms = bms / max(bcnt, 1)
        bwd_bytes = _render_bwd_alg_bytes(P_vis / B, W, H) * B
        bwd_ach = bwd_bytes / (bwd_ms * 1e-3) / 1e9 if bwd_ms > 0 else None
        out["roofline_bwd"] = {"bound": "hbm", "kernel": "render_bwd",
                               "achieved": round(bwd_ach, 1) if bwd_ach else None, "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(bwd_ach / HBM_PEAK_GBS, 4) if bwd_ach else None,
                               "traffic": bwd_traffic, "alg_bytes_per_launch": bwd_bytes,
                               "avg_launch_ms": round(bwd_ms, 4), "us_per_frame": round(1000 * bwd_ms / B, 2)}
    if a.pipeline == "frame":
        out["latency_ms_per_frame"] = round(1000.0 * el / (a.steps * B), 4)
    if deform_ms is not None:
        out["deform_ms_per_step"] = round(deform_ms, 4)
    if exact_line is not None:
        out["exact_accum"] = exact_line
    if a.stages:
        out["stage_ms_per_step"] = {k: round(v[0] / max(v[1], 1), 4) for k, v in prof.items()}
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.pipeline != "train":
        out["cpu_baseline"] = cpu_baseline(scene, cams, W, H, a.cpu_seconds, avatar_inputs)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
