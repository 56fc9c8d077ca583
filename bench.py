#!/usr/bin/env python
"""Headline benchmark: rendered frames/sec at 512x512 with ~100k Gaussians (BASELINE.json).

One step = one pass of GUAVA's per-frame animation path over a batch of tracked frames
(config 2 "self-reenactment": main/test.py:70-76 times Ubody_Gaussian.forward + render per frame):
  --pipeline avatar (default): EHM deformation (FLAME head LBS + SMPL-X body LBS, per-frame pose,
      expression, eyelids), vertex + UV Gaussian assembly, then the rasterizer hot path
      (preprocess -> tile binning -> per-tile depth order -> 32-channel compositing);
      --config c5: 300k Gaussians (3 per UV texel), 1024x1024, cross-reenactment poses
      (main/test.py:96-139: target poses with the source identity);
  --pipeline raster: the rasterizer alone over one static cloud seen by a camera per frame;
  --pipeline train: BASELINE config 4 (raster fwd + fused-SSIM/L1 loss + raster bwd + Adam);
  --pipeline frame: GUAVA's unchanged caller, GaussianRasterizer_32 once per frame.
Synthetic avatar: P=100,000 Gaussians (10,475 SMPL-X vertex Gaussians + UV Gaussians), 512x512,
one camera and one pose per frame; every input resident in HBM before the timed region.

Numerics: the headline is the bit-exact f32 path (colour accumulation on f32 MFMAs, identical to
the CPU oracle); --split-bf16 measures the tolerance mode instead (the line then carries the f32
number under `exact_accum`); by default the split-bf16 number is an extra key (`split_bf16`).

N GPUs: one process per GPU.  `--gpus N` starts the N ranks itself (torch.distributed.run, before
anything touches the GPU) unless it already runs under a launcher (WORLD_SIZE set, which must
equal N).  Frames are sharded over ranks: by default each rank renders its own `--batch` frames
("scaling": "weak"); `--global-batch G` splits G frames over the ranks instead ("strong"; config 3
is G=32 over 8 GPUs).  Every step ends with the consumer exchange: the rendered frames are encoded
as GUAVA's 8-bit RGB (to8b, main/test.py:85) and all-gathered over RCCL/xGMI to every rank,
overlapped with the next step's rendering (the timed region ends after the last exchange).  The
line's time is the max over ranks.

Prints ONE JSON line (rank 0) with the contract fields plus:
  roofline        -- render_fwd kernel: algorithmic bytes per launch / average launch time from HIP
                     events recorded on the launch stream inside the timed region; `traffic` from the
                     committed PMC summary only when it was measured on this build (source hash);
  cpu_baseline    -- the CPU oracle (a port of the reference algorithm) timed on a bounded sample of
                     the same workload on this host's cores (rank 0, N=1 only);
  per_frame_dropin-- GUAVA's own fps definition (main/test.py:70-76,90): deform + one
                     GaussianRasterizer_32 call per frame, B=1 (N=1 only);
  config3_strong  -- at N>1: config 3 itself, 32 frames per step split over the N ranks.
"""
import argparse
import json
import os
import socket
import subprocess
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
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per step per GPU (weak scaling; default 32, 6 for --pipeline train)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="frames per step over ALL ranks (strong scaling; config 3 = 32 over 8 GPUs)")
    ap.add_argument("--config", default="c2", choices=["c2", "c5"])
    ap.add_argument("--pipeline", default="avatar", choices=["avatar", "raster", "train", "frame"],
                    help="train = BASELINE config 4: raster fwd + fused-SSIM/L1 loss + raster bwd + "
                         "gradient all-reduce + Adam; frame = GUAVA's unchanged caller: "
                         "one GaussianRasterizer_32 call per frame as gaussian_render.py:37-67 does")
    ap.add_argument("--inflight", type=int, default=None,
                    help="batches in flight on separate HIP streams (avatar/raster pipelines; default 4 at c2, "
                         "2 at the render-bound c5: the deform + binning chains of the next batches run beside "
                         "one batch's compositing; at N>1 at most GPU_MAX_HW_QUEUES - 1, parallel.stream_budget); "
                         "kernel times for the roofline then come from an isolated pass")
    ap.add_argument("--refine", action="store_true",
                    help="fuse the refiner's first 1x1 conv 32->16 + leaky ReLU into the render "
                         "epilogue (inference output: 16 refiner features + 4 raw channels)")
    ap.add_argument("--fast-exp", action="store_true", help="hardware exp (not bit-exact)")
    ap.add_argument("--split-bf16", action="store_true",
                    help="headline in the split-bf16 colour-accumulation mode (tolerance, include/gsr.h)")
    ap.add_argument("--gather", default="u8", choices=["u8", "f32", "none"],
                    help="N>1 consumer exchange: 8-bit RGB (to8b, default), f32 RGB, or none")
    ap.add_argument("--cu-split", type=int, default=None,
                    help="render placement (include/gsr.h gsr_set_render_stream): the batches' deform + binning "
                         "chains on streams masked to this many CUs, every compositing kernel on one render "
                         "stream masked to the other CUs (0: the same routing without masks)")
    ap.add_argument("--cu-mode", default="spread", choices=["spread", "lo"],
                    help="which CUs the --cu-split slice takes (parallel.cu_masks)")
    ap.add_argument("--render-streams", type=int, default=0,
                    help="route the compositing kernels of the batches' streams to this many render streams "
                         "(include/gsr.h gsr_set_render_stream; 0: each batch renders on its own stream)")
    ap.add_argument("--prep-priority", type=int, default=0,
                    help="HIP stream priority of the batches' streams when --render-streams is set "
                         "(torch convention: lower is higher priority; the render streams keep 0)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="only the contract measurement (no split-bf16 / per-frame / config-3 extras)")
    ap.add_argument("--stages", action="store_true", help="also time every stage (extra events)")
    a = ap.parse_args()
    if a.batch is None:
        a.batch = 6 if a.pipeline == "train" else 32
    if a.inflight is None:
        a.inflight = 2 if a.config == "c5" else 4
    return a


def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process -- nothing here has touched the GPU -- and exit with
    its status.  Rank 0's JSON line reaches stdout through the child."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


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


class Workload:
    """The synthetic inputs and the per-step callable of one pipeline for B frames of this rank
    (frames [lo, hi) of n_total), resident in HBM."""

    def __init__(self, a, wl, B, lo, n_total, dev, numerics):
        import torch
        from guava_renderer_amd import scenes
        from guava_renderer_amd.batch import BatchRasterizer
        self.a, self.B, self.dev = a, B, dev
        P, W, H = wl["P"], wl["W"], wl["H"]
        self.W, self.H = W, H
        cams_all = scenes.frame_cameras(n_total, W, H, seed=1000)
        self.cams = cams = cams_all[lo:lo + B]
        t = lambda x: torch.tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
        self.t = t
        views = t(np.stack([c["viewmatrix"].reshape(16) for c in cams]))
        projs = t(np.stack([c["projmatrix"].reshape(16) for c in cams]))
        tanf = t(np.array([[c["tanfovx"], c["tanfovy"]] for c in cams], np.float32))
        self.views, self.projs, self.tanf = views, projs, tanf
        bgs = torch.zeros((B, C), dtype=torch.float32, device=dev)
        self.avatar_inputs = None
        self.rasts = []
        self.pipes = []
        self.trainer = None
        if a.pipeline in ("avatar", "frame"):
            from guava_renderer_amd import avatar
            from guava_renderer_amd.pipeline import AvatarPipeline
            body, flame, extra = avatar.ehm_assets(seed=0)
            verts, faces, tex = avatar.template_mesh()
            g = avatar.gaussians(verts, faces, tex * wl["gpt"], P=P, seed=0)
            bp_all, fp_all = avatar.ehm_params(n_total, seed=1000)
            if a.config == "c5":  # cross-reenactment: target poses on the source identity
                src_b, src_f = avatar.ehm_params(1, seed=77)
                bp_all, fp_all = avatar.change_id_info(bp_all, fp_all, src_b, src_f)
            bp = {k: v[lo:lo + B] for k, v in bp_all.items()}
            fp = {k: v[lo:lo + B] for k, v in fp_all.items()}
            self.bpt = {k: t(v) for k, v in bp.items()}
            self.fpt = {k: t(v) for k, v in fp.items()}
            self.avatar_assets = (body, flame, extra, g)
            self.avatar_inputs = (body, flame, extra, g, bp, fp)
            self.scene = {"colors": g["colors"], "opacities": g["opacities"]}
            probe = AvatarPipeline(body, flame, extra, g, B, W, H, R_capacity=24 * P * B, device=dev)
            self.P = probe.P
            if a.pipeline == "avatar":
                probe.render(self.bpt, self.fpt, views, projs, tanf)
                R_probe, ovf = probe.rast.status()
                assert not ovf, "probe overflow"
                del probe
                torch.cuda.empty_cache()
                self.pipes = [AvatarPipeline(body, flame, extra, g, B, W, H, R_capacity=int(R_probe * 1.25) + 1024,
                                             device=dev) for _ in range(max(1, a.inflight))]
                for p in self.pipes:
                    p.rast.numerics = numerics
                self.rasts = [p.rast for p in self.pipes]
                head = None
                if a.refine:
                    from guava_renderer_amd.batch import RefineHead
                    rng = np.random.default_rng(5)  # random-init conv_body_first (nn.Conv2d(32, 16, 1))
                    head = RefineHead(t(rng.uniform(-0.18, 0.18, (16, 32)).astype(np.float32)),
                                      t(rng.uniform(-0.18, 0.18, 16).astype(np.float32)), keep_channels=4)
                pipes = self.pipes
                # fused: Gaussian assembly inside the projection kernel (gsr_forward_batch_deformed);
                # no refiner epilogue on that entry, so --refine keeps the two-step path
                fused = head is None and os.environ.get("GSR_AVATAR_FUSED", "0") == "1"
                self.config_extra = {"fused_deform": fused}
                self.step_on = lambda i: pipes[i].render(self.bpt, self.fpt, views, projs, tanf, refine=head,
                                                         fused=fused)
            else:
                self._frame_pipeline(probe, numerics)
        elif a.pipeline == "train":
            from guava_renderer_amd.train import SplatTrainer
            scene = scenes.avatar_cloud(P, seed=0, gaussians_per_texel=wl["gpt"])
            self.scene = scene
            self.P = P = scene["means3D"].shape[0]
            params = {k: t(scene[k]) for k in ("means3D", "colors", "opacities", "scales", "rotations")}
            probe = BatchRasterizer(B, P, W, H, R_capacity=24 * P * B, device=dev)
            probe.forward(params["means3D"], params["colors"], params["opacities"], params["scales"],
                          params["rotations"], views, projs, tanf, bgs)
            R_probe, ovf = probe.status()
            assert not ovf, "probe overflow"
            del probe
            torch.cuda.empty_cache()
            # the trainable parameters are the raw attributes: a small learning
            # rate keeps the per-step work at the avatar's distribution over the timed steps;
            # capacity with headroom for the drift (an overflowing step is skipped on the device)
            self.trainer = SplatTrainer(params, B, W, H, R_capacity=int(R_probe * 2) + 1024, device=dev, lr=1e-5,
                                        numerics=numerics)
            self.rasts = [self.trainer.rast]
            target = torch.rand((B, 3, H, W), device=dev, generator=torch.Generator(device=dev).manual_seed(lo))
            self.step_on = lambda i: self.trainer.step(views, projs, tanf, target)
        else:
            scene = scenes.avatar_cloud(P, seed=0, gaussians_per_texel=wl["gpt"])
            self.scene = scene
            self.P = P = scene["means3D"].shape[0]
            means, colors = t(scene["means3D"]), t(scene["colors"])
            opac, scales, rots = t(scene["opacities"]), t(scene["scales"]), t(scene["rotations"])
            probe = BatchRasterizer(B, P, W, H, R_capacity=24 * P * B, device=dev)
            probe.forward(means, colors, opac, scales, rots, views, projs, tanf, bgs)
            R_probe, ovf = probe.status()
            assert not ovf, "probe overflow"
            del probe
            torch.cuda.empty_cache()
            self.rasts = [BatchRasterizer(B, P, W, H, R_capacity=int(R_probe * 1.25) + 1024, device=dev,
                                          numerics=numerics) for _ in range(max(1, a.inflight))]
            rasts = self.rasts
            self.step_on = lambda i: rasts[i].forward(means, colors, opac, scales, rots, views, projs, tanf, bgs,
                                                      forward_only=True)
        self.rast = self.rasts[0] if self.rasts else None

    def _frame_pipeline(self, dpipe, numerics):
        """GUAVA's unchanged caller (models/UbodyAvatar/gaussian_render.py:19-67, the refiner aside):
        one GaussianRasterizationSettings + GaussianRasterizer_32 call per frame, camera fields read
        per frame with int()/float() from device tensors, outputs stacked.  The deformed assets of
        the B frames come from the deform kernels, outside the timed region."""
        import torch
        from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32
        B, dev, H, W = self.B, self.dev, self.H, self.W
        dg = dpipe.deform(self.bpt, self.fpt)
        assets = {"xyz": dg["xyz"], "rotation": dg["rotation"], "scaling": dg["scaling"],
                  "opacity": dpipe.gauss.opacity.unsqueeze(0).expand(B, -1, -1),
                  "features_color": dpipe.gauss.colors.unsqueeze(0).expand(B, -1, -1)}
        cam_params = _cam_params(self, B)
        self.last_radii = [None]

        def step_on(i):
            with torch.no_grad():
                out, radii, depths = _render_model(assets, cam_params, B, dev, GaussianRasterizationSettings,
                                                   GaussianRasterizer_32)
                self.last_radii[0] = radii
                return out, depths, radii
        self.step_on = step_on


def _cam_params(w, B, lo=0):
    """render_cam_params of B frames as GUAVA's data loader hands them to GaussianRenderer
    (dataset/data_loader.py:232-251): device tensors, one row per frame."""
    import torch
    sl = slice(lo, lo + B)
    return {"image_height": torch.full((B,), w.H, device=w.dev), "image_width": torch.full((B,), w.W, device=w.dev),
            "tanfovx": w.tanf[sl, 0].contiguous(), "tanfovy": w.tanf[sl, 1].contiguous(),
            "world_view_transform": w.views[sl].view(B, 4, 4), "full_proj_transform": w.projs[sl].view(B, 4, 4),
            "camera_center": w.t(np.stack([c["campos"] for c in w.cams[sl]]))}


def _render_model(assets, cam_params, B, dev, Settings, Rasterizer):
    """GaussianRenderer.forward's rasterizer loop (gaussian_render.py:19-67) as GUAVA runs it."""
    import torch
    mean_3d = assets["xyz"]
    features_color = assets["features_color"].clone()
    mean_2d = torch.zeros_like(mean_3d, dtype=torch.float32, requires_grad=True, device=dev)
    bg = torch.ones((B, features_color.shape[-1]), dtype=torch.float32, device=dev) * 0.0
    imgs, radiis, depths = [], [], []
    for bi in range(B):
        rs = Settings(
            image_height=int(cam_params["image_height"][bi]), image_width=int(cam_params["image_width"][bi]),
            tanfovx=float(cam_params["tanfovx"][bi]), tanfovy=float(cam_params["tanfovy"][bi]),
            bg=bg[bi], scale_modifier=1.0, viewmatrix=cam_params["world_view_transform"][bi],
            projmatrix=cam_params["full_proj_transform"][bi], sh_degree=0,
            campos=cam_params["camera_center"][bi], prefiltered=False, debug=False, antialiasing=False)
        img, rad, dep = Rasterizer(raster_settings=rs)(
            means3D=mean_3d[bi], means2D=mean_2d[bi], shs=None, colors_precomp=features_color[bi],
            opacities=assets["opacity"][bi], scales=assets["scaling"][bi],
            rotations=assets["rotation"][bi], cov3D_precomp=None)
        imgs.append(img)
        radiis.append(rad)
        depths.append(dep)
    return torch.stack(imgs, 0), torch.stack(radiis, 0), torch.stack(depths, 0)


def per_frame_dropin(w, dev, n_frames=256, warmup=16):
    """GUAVA's own fps (main/test.py:70-76,90): per frame, Ubody_Gaussian.forward (here the deform
    kernels at B=1) then GaussianRenderer's rasterizer call through the unchanged drop-in API
    (GaussianRasterizer_32, gaussian_render.py:37-67), B=1, under no_grad as render_set runs.
    fps = frames / wall time of the loop (the int()/float() camera reads serialise the frames as
    they do in the reference); the loop ends with a device synchronisation."""
    import torch
    from diff_gaussian_rasterization_32 import GaussianRasterizationSettings, GaussianRasterizer_32
    from guava_renderer_amd.pipeline import AvatarPipeline
    body, flame, extra, g = w.avatar_assets
    pipe = AvatarPipeline(body, flame, extra, g, 1, w.W, w.H, R_capacity=1024, device=dev)
    frames = [({k: v[i:i + 1] for k, v in w.bpt.items()}, {k: v[i:i + 1] for k, v in w.fpt.items()},
               _cam_params(w, 1, lo=i)) for i in range(w.B)]
    opacity = pipe.gauss.opacity.unsqueeze(0)
    colors = pipe.gauss.colors.unsqueeze(0)

    def frame(k):
        bp, fp, cam = frames[k % len(frames)]
        dg = pipe.deform(bp, fp)  # Ubody_Gaussian.forward (ubody_gaussian.py:245-289)
        assets = {"xyz": dg["xyz"], "rotation": dg["rotation"], "scaling": dg["scaling"],
                  "opacity": opacity, "features_color": colors}
        return _render_model(assets, cam, 1, dev, GaussianRasterizationSettings, GaussianRasterizer_32)

    with torch.no_grad():
        for k in range(warmup):
            frame(k)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(n_frames):
            frame(k)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
    return {"value": round(n_frames / el, 2), "unit": "frames/s", "latency_ms_per_frame": round(1e3 * el / n_frames, 4),
            "frames": n_frames, "batch": 1,
            "path": "deform (B=1) + GaussianRasterizer_32 per frame, no_grad (main/test.py:70-76)"}


def config_line(a, config, pipeline, dev, numerics, steps, warmup=5):
    """One of BASELINE.json's other single-GPU configurations as an extra line of the default run
    (N=1): config 4 (pipeline "train": batch 6, raster fwd + fused-SSIM/L1 loss + raster bwd + Adam)
    or config 5 (config "c5": 300k Gaussians, 1024x1024, cross-reenactment deform + raster, two
    batches in flight).  Same timing method as the contract line (wall clock over `steps` steps
    between device synchronisations); the render kernels' launch times come from HIP events on the
    launch stream (a separate isolated pass when batches overlap)."""
    import copy
    import torch
    from guava_renderer_amd.batch import profile_enable, profile_read
    b = copy.copy(a)
    b.config, b.pipeline = config, pipeline
    b.batch = 6 if pipeline == "train" else 32
    b.inflight = 1 if pipeline == "train" else (2 if config == "c5" else 4)
    b.refine = False
    wl = _workload(config)
    W, H, B = wl["W"], wl["H"], b.batch
    w = Workload(b, wl, B, 0, B, dev, numerics)
    n_in = max(1, len(w.rasts)) if pipeline != "train" else 1
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(n_in - 1)]
    cnt = [0]

    def step():
        i = cnt[0] % n_in
        cnt[0] += 1
        with torch.cuda.stream(streams[i]):
            return w.step_on(i)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    stages = ("render_fwd", "render_bwd") if pipeline == "train" else ("render_fwd",)
    profile_read()
    profile_enable(stages if n_in == 1 else ())
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    prof = profile_read()
    profile_enable(())
    if n_in > 1:  # kernel times from an isolated pass (one batch at a time)
        profile_enable(stages)
        for _ in range(max(10, steps // 2)):
            w.step_on(0)
        torch.cuda.synchronize(dev)
        prof = profile_read()
        profile_enable(())
    if pipeline == "train":
        assert w.trainer.skipped_steps == 0, "capacity overflow inside the timed region"
    else:
        assert not any(r.status()[1] for r in w.rasts), "capacity overflow inside the timed region"
    P_vis = int((w.rast.radii > 0).sum().item())
    out = {"value": round(B * steps / el, 2), "unit": "frames/s", "ms_per_step": round(1e3 * el / steps, 4),
           "steps": steps, "frames_per_step": B, "batches_in_flight": n_in,
           "workload": wl["name"] + ("-train" if pipeline == "train" else "-deform+raster-cross"),
           "gaussians": w.P, "image": [W, H], "visible_gaussians_per_frame": P_vis / B}
    rms, rc = prof.get("render_fwd", (0.0, 0))
    if rc:
        ms = rms / rc
        ab = _render_alg_bytes(P_vis / B, W, H) * B
        out["roofline"] = {"kernel": "render_fwd", "avg_launch_ms": round(ms, 4), "alg_bytes_per_launch": ab,
                           "achieved": round(ab / (ms * 1e-3) / 1e9, 1),
                           "frac": round(ab / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    bms, bc = prof.get("render_bwd", (0.0, 0))
    if bc:
        ms = bms / bc
        ab = _render_bwd_alg_bytes(P_vis / B, W, H) * B
        out["roofline_bwd"] = {"kernel": "render_bwd", "avg_launch_ms": round(ms, 4), "alg_bytes_per_launch": ab,
                               "us_per_frame": round(1e3 * ms / B, 2),
                               "achieved": round(ab / (ms * 1e-3) / 1e9, 1),
                               "frac": round(ab / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        pmc = os.path.join(ROOT, "profiles", "pmc_train.json")
        try:
            from guava_renderer_amd import build as _build
            pm = json.load(open(pmc))
            if pm.get("source_hash") == _build.source_hash() and pm.get("batch") == B:
                out["roofline_bwd"]["traffic"] = (pm.get("kernels", {}).get("k_render_bwd") or {}).get("hbm_bytes")
                out["roofline_bwd"]["traffic_source"] = "PMC FETCH_SIZE+WRITE_SIZE, pmc_train.json (this build)"
        except (OSError, ValueError):
            pass
    del w
    torch.cuda.empty_cache()
    return out


def main():
    a = _args()
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and a.gpus > 1:
        sys.exit(_launch_ranks(a.gpus))
    world = int(ws or "1")
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    import torch
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

    from guava_renderer_amd import _lib, parallel
    from guava_renderer_amd.batch import profile_enable, profile_read, render_counters

    numerics = _lib.numerics(fast_exp=a.fast_exp, split_bf16=a.split_bf16)
    wl = _workload(a.config)
    W, H = wl["W"], wl["H"]
    if a.global_batch is not None:
        if a.global_batch % world:
            print(f"bench.py: --global-batch {a.global_batch} does not split over {world} ranks", file=sys.stderr)
            sys.exit(2)
        B, scaling, n_total = a.global_batch // world, "strong", a.global_batch
    else:
        B, scaling, n_total = a.batch, "weak", a.batch * world
    lo = rank * B
    # hardware-queue budget: at N>1 one of the GPU_MAX_HW_QUEUES queues stays free for RCCL
    a.inflight = parallel.stream_budget(a.inflight, world)
    w = Workload(a, wl, B, lo, n_total, dev, numerics)
    P = w.P
    workload = wl["name"] + {"avatar": "-deform+raster" + ("-cross" if a.config == "c5" else ""),
                             "raster": "-raster", "train": "-train", "frame": "-per-frame-dropin"}[a.pipeline]

    # batches in flight: step k runs on stream k mod n with its own pipeline / workspace (each
    # batch is complete work -- deform, binning, compositing; only consecutive batches overlap)
    n_inflight = max(1, len(w.rasts))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(n_inflight - 1)]
    placement = None
    if a.cu_split is not None and a.pipeline in ("avatar", "raster"):
        placement = parallel.SplitPlacement(n_inflight, a.cu_split, dev, mode=a.cu_mode)
        streams = placement.streams
    elif a.render_streams > 0 and a.pipeline in ("avatar", "raster"):
        streams = [torch.cuda.Stream(dev, priority=a.prep_priority) for _ in range(n_inflight)]
        rstreams = [torch.cuda.Stream(dev) for _ in range(a.render_streams)]
        for i, st in enumerate(streams):
            _lib.check(_lib.load().gsr_set_render_stream(st.cuda_stream, rstreams[i % len(rstreams)].cuda_stream),
                       "gsr_set_render_stream")

    # consumer boundary at N>1: every rank receives all ranks' frames as the consumer writes them
    # (8-bit RGB, main/test.py:85) over RCCL/xGMI, each batch's exchange overlapped with the next
    # batch's rendering on a side stream
    def make_gatherer(b):
        if dist is None or a.pipeline == "train" or a.gather == "none":
            return None
        gdev = dev if backend == "nccl" else torch.device("cpu")
        return parallel.FrameGather(b, (3, H, W), torch.uint8 if a.gather == "u8" else torch.float32, gdev)

    def make_step(wk, gatherer, inflight=None):
        cnt = [0]
        nin = n_inflight if inflight is None else inflight

        def step():
            i = cnt[0] % nin
            cnt[0] += 1
            with torch.cuda.stream(streams[i]):
                res = wk.step_on(i)
                if gatherer is not None:
                    frames = res[0]
                    if backend != "nccl":  # gloo rehearsal: encode on the GPU, exchange on the host
                        frames = parallel.frames_to8b(frames).cpu() if a.gather == "u8" else frames[:, :3].cpu()
                    elif a.gather == "f32":
                        frames = frames[:, :3]
                    gatherer.push(frames)
                return res
        return step

    def timed(step, gatherer, steps, warmup):
        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        if gatherer is not None:
            gatherer.wait()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if dist is not None:
            dist.barrier()
            tt = torch.tensor([el], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el

    gatherer = make_gatherer(B)
    step = make_step(w, gatherer)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if w.rast is not None:
        R_total, ovf = w.rast.status()
        assert not any(r.status()[1] for r in w.rasts)
        P_vis = int((w.rast.radii > 0).sum().item())
    else:  # per-frame drop-in path: the _C calls size their own buffers
        R_total = None
        P_vis = int((w.last_radii[0] > 0).sum().item())
    profile_read()  # reset accumulators
    stage_set = (("preprocess", "scan", "depth_sort", "chunk_count", "tile_scan", "ordered_scatter",
                  "render_fwd", "render_bwd", "preprocess_bwd") if a.stages else
                 ("render_fwd", "render_bwd") if a.pipeline == "train" else ("render_fwd",))
    # with batches overlapping, a kernel's event-timed duration includes the other batch's work:
    # the timed region then carries no stage events, and the kernel times (roofline) come from an
    # isolated pass afterwards, one batch at a time
    isolated = n_inflight > 1
    profile_enable(() if isolated else stage_set)
    el = timed(step, gatherer, a.steps, 0)
    prof = profile_read()
    profile_enable(())
    if isolated:
        profile_enable(stage_set)
        for _ in range(max(20, a.steps // 4)):
            with torch.cuda.stream(streams[0]):
                w.step_on(0)
        torch.cuda.synchronize(dev)
        prof = profile_read()
        profile_enable(())
    if a.pipeline == "train":
        assert w.trainer.skipped_steps == 0 and not w.trainer.rast.status()[1], \
            "capacity overflow inside the timed region"
    else:
        assert not any(r.status()[1] for r in w.rasts), "capacity overflow inside the timed region"
    extras = not a.no_extras
    deform_ms = None
    if a.pipeline == "avatar":  # deformation alone (EHM + Gaussian assembly), outside the timed region
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            w.pipes[0].deform(w.bpt, w.fpt)
        e1.record()
        torch.cuda.synchronize(dev)
        deform_ms = e0.elapsed_time(e1) / a.steps
    # the other colour-accumulation mode on the same workload, a shorter run after the timed region
    other_line = None
    if extras and dist is None and a.pipeline in ("avatar", "raster"):
        other = numerics ^ _lib.NUMERICS_SPLIT_BF16
        for r in w.rasts:
            r.numerics = other
        n_o = max(20, a.steps // 4)
        el_o = timed(step, None, n_o, 3)
        for r in w.rasts:
            r.numerics = numerics
        other_line = {"value": round(B * n_o / el_o, 2), "ms_per_step": round(1e3 * el_o / n_o, 4), "steps": n_o,
                      "colour_accum": "split-bf16 mfma (<=1e-4 L_inf)" if other & _lib.NUMERICS_SPLIT_BF16
                      else "f32 mfma (bit-exact with the oracle)"}
    # the same workload with one batch in flight (kernel-level gain vs overlap gain, same process)
    one_line = None
    if extras and dist is None and n_inflight > 1 and a.pipeline in ("avatar", "raster"):
        n_1 = max(20, a.steps // 4)
        el_1 = timed(make_step(w, None, inflight=1), None, n_1, 3)
        one_line = {"value": round(B * n_1 / el_1, 2), "ms_per_step": round(1e3 * el_1 / n_1, 4), "steps": n_1,
                    "batches_in_flight": 1}
    # work counters of one extra (instrumented, untimed) step: which wall the render kernel hits
    work = render_counters(step, device=dev)
    # config 3 at N>1: the 32-frame batch split over the ranks (strong scaling) beside the weak line
    strong_line = None
    if extras and dist is not None and scaling == "weak" and a.pipeline == "avatar" and 32 % world == 0:
        w3 = Workload(a, wl, 32 // world, rank * (32 // world), 32, dev, numerics)
        g3 = make_gatherer(32 // world)
        n3 = max(20, a.steps // 4)
        el3 = timed(make_step(w3, g3), g3, n3, 5)
        strong_line = {"value": round(32 * n3 / el3, 2), "ms_per_step": round(1e3 * el3 / n3, 4), "steps": n3,
                       "global_batch": 32, "frames_per_gpu": 32 // world, "scaling": "strong"}
        del w3, g3

    frames = world * B * a.steps
    fps = frames / el
    ms_step = 1000.0 * el / a.steps
    rms, rcnt = prof.get("render_fwd", (0.0, 0))
    render_ms = rms / max(rcnt, 1)
    frames_per_launch = 1 if a.pipeline == "frame" else B
    bytes_launch = _render_alg_bytes(P_vis / B, W, H) * frames_per_launch
    achieved = bytes_launch / (render_ms * 1e-3) / 1e9 if render_ms > 0 else None
    traffic = issue = bwd_traffic = None
    traffic_note = "no PMC summary for this workload"
    # HBM traffic per launch from the committed PMC summaries (tools/pmc_summary.py), used only when
    # they were measured on the library built from these sources (their source hash)
    pmc_path = os.path.join(ROOT, "profiles", "pmc_train.json" if a.pipeline == "train" else "pmc_render_fwd.json")
    if os.path.exists(pmc_path):
        try:
            from guava_renderer_amd import build as _build
            pm = json.load(open(pmc_path))
            if pm.get("config") == workload and pm.get("batch") == B:
                if pm.get("source_hash") == _build.source_hash():
                    traffic = pm.get("hbm_bytes_per_launch")
                    issue = pm.get("render_fwd_issue")
                    bwd_traffic = (pm.get("kernels", {}).get("k_render_bwd") or {}).get("hbm_bytes")
                    traffic_note = f"PMC FETCH_SIZE+WRITE_SIZE, {os.path.basename(pmc_path)} (this build)"
                else:
                    traffic_note = f"{os.path.basename(pmc_path)} was measured on another build: not used"
        except Exception as e:  # noqa: BLE001
            traffic_note = f"PMC summary unreadable: {e}"

    split_head = bool(numerics & _lib.NUMERICS_SPLIT_BF16)
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
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32 (colour products in split-bf16: f = f_hi + f_lo, f32 accumulation)" if split_head else "f32",
        "data": ("synthetic avatar (SMPL-X template mesh + UV-texel Gaussians, synthetic LBS bases, "
                 "GUAVA attribute distributions), one pose + one orbit camera per frame"
                 + (", cross-reenactment (target poses, source identity)" if a.config == "c5" else "")
                 if a.pipeline in ("avatar", "frame") else
                 "synthetic (SMPL-X-template avatar cloud, GUAVA attribute distributions, "
                 "one orbit camera per frame)"),
        "config": {"workload": workload,
                   "pipeline": {"avatar": "EHM LBS -> Gaussian assembly -> rasterize",
                                "raster": "rasterize",
                                "train": "raster fwd -> L1 + fused SSIM (raw RGB) + L1 of a fixed 32->3 refine stand-in "
                                         "(all 32 channels carry gradient) -> frame-reduced raster bwd -> "
                                         "grad all-reduce -> Adam",
                                "frame": "deformed frames -> GaussianRasterizer_32 once per frame (gaussian_render.py:37-67)"
                                }[a.pipeline] + (" + fused refiner conv_body_first" if a.refine else "")
                               + (" (assembly fused into the projection kernel)"
                                  if getattr(w, "config_extra", {}).get("fused_deform") else ""),
                   "gaussians": P, "image": [W, H], "channels": C,
                   "frames_per_step_per_gpu": B, "global_batch": B * world,
                   "parallelism": f"frame-sharded x{world}" + (
                       f", {a.gather} RGB all-gather per step (overlapped with the next step)"
                       if world > 1 and a.pipeline != "train" and a.gather != "none" else
                       ", gradient all-reduce per step" if world > 1 and a.pipeline == "train" else ""),
                   "batches_in_flight": n_inflight,
                   "placement": ({"prep_cus": placement.prep_cus, "render_cus": placement.render_cus,
                                  "mode": placement.mode} if placement is not None else
                                 {"render_streams": a.render_streams, "prep_priority": a.prep_priority}
                                 if a.render_streams > 0 else "shared"),
                   "exp": "hw" if a.fast_exp else "exact-poly",
                   "colour_accum": "split-bf16 mfma (<=1e-4)" if split_head else "f32 mfma (bit-exact)",
                   "instances_per_step": R_total, "visible_gaussians_per_frame": P_vis / B},
        "roofline": {"bound": "hbm", "kernel": "render_fwd",
                     "achieved": round(achieved, 1) if achieved else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "traffic_source": traffic_note, "alg_bytes_per_launch": bytes_launch,
                     "avg_launch_ms": round(render_ms, 4),
                     "timing": "isolated pass, one batch in flight" if isolated else "timed region"},
        "path_roofline": {"alg_bytes_per_frame": _path_alg_bytes(P, W, H),
                          "achieved_GBs": round(_path_alg_bytes(P, W, H) * fps / 1e9, 1),
                          "frac": round(_path_alg_bytes(P, W, H) * fps / 1e9 / HBM_PEAK_GBS, 4)},
    }
    # per-frame work of the render kernel and its matrix-core utilisation (dense peak of the MFMA used)
    ksteps = work["mfma_ksteps"]
    if not split_head:
        mfma_flops = ksteps * 2 * (2 * 32 * 32 * 2)  # two v_mfma_f32_32x32x2f32 per wave k-step
    else:  # two v_mfma_f32_32x32x8_bf16 per wave k-step (every k-slot carries a split product)
        mfma_flops = ksteps * 2 * (2 * 32 * 32 * 8)
    out["render_work_per_frame"] = {k: round(v / B, 1) for k, v in work.items()}
    out["render_mfma"] = {"issued_tflops": round(mfma_flops / (render_ms * 1e-3) / 1e12, 2) if render_ms else None,
                          "peak_tflops": BF16_MFMA_PEAK_TFLOPS if split_head else F32_MFMA_PEAK_TFLOPS,
                          "instruction": "v_mfma_f32_32x32x8_bf16" if split_head else "v_mfma_f32_32x32x2_f32",
                          # lane-pairs blended: 64 pixels per survivor in the strip layout
                          "useful_frac": round(work["pairs_contributing"] / max(64 * work["strip_pairs_blended"], 1),
                                               4)}
    if issue is not None:
        # the compute wall beside the HBM one: per-launch instruction counts and per-SIMD pipe busy
        # of the contract kernel, from the committed PMC passes of this build
        out["render_issue"] = dict(issue, source="profiles/pmc_render_fwd.json (tools/gpu_pmc.sh)",
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
    if other_line is not None:
        out["split_bf16" if not split_head else "exact_accum"] = other_line
    if strong_line is not None:
        out["config3_strong"] = strong_line
    if one_line is not None:
        out["one_in_flight"] = one_line
    if a.stages:
        out["stage_ms_per_step"] = {k: round(v[0] / max(v[1], 1), 4) for k, v in prof.items()}
    if extras and world == 1 and a.pipeline == "avatar":
        out["per_frame_dropin"] = per_frame_dropin(w, dev)
    if extras and world == 1 and a.pipeline == "avatar" and a.config == "c2":
        # BASELINE configs 4 and 5 on one GPU, beside the contract line (their N>1 forms are the
        # driver's multi-GPU runs: --pipeline train / --config c5 with --gpus N)
        out["config4_train"] = config_line(a, "c2", "train", dev, numerics, steps=max(a.steps, 100))
        out["config5_cross"] = config_line(a, "c5", "avatar", dev, numerics, steps=max(a.steps, 40))
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.pipeline != "train":
        out["cpu_baseline"] = cpu_baseline(w.scene, w.cams, W, H, a.cpu_seconds, w.avatar_inputs)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
