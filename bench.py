#!/usr/bin/env python3
"""Throughput of the embed + match hot path (BASELINE.json metric), one JSON line.

Workload at N=1 (BASELINE.json configs[2]): IR-101 AdaFace embed + cosine top-5
match of a batch of 256 synthetic 112x112 crops per GPU against a 1k-row
gallery.  One "step" = one ``fr_embed_match`` over the rank's batch, inputs
already resident in HBM.  For N>1 there is one rank per GPU: ``--gpus N`` starts
the N rank processes itself (fresh children, before this process touches the
GPU), or runs as one of them under ``torchrun`` (WORLD_SIZE set; ``--gpus``
may then be omitted, and must equal WORLD_SIZE when given).  Rank 0 embeds the gallery and broadcasts it over RCCL (the path's
only exchange step); each rank then processes its own probes independently
(weak scaling: N x batch faces per step).

Also reported:
  roofline      the dominant conv kernel family (wino4_kernel for the stride-1 3x3 convs
                under the f32 default): algorithmic (direct-conv) FLOP / summed
                HIP-event time of its launches, vs the 157.3 TF dense fp32 MFMA
                peak; executed_* counts the MFMA work Winograd actually performs.
                The events are recorded in a second timed pass of the same K steps
                (ms_per_step_profiled_pass): an event pair around every launch adds
                ~0.8 ms per IR-101 step, so the throughput pass runs without them.
  gallery_exchange (N > 1)  the broadcast's bytes, ms (first, and median of
                --exchange-reps repeats) and GB/s, max over ranks; plus the fastest and
                slowest rank's ms/step (rank_ms_per_step_min/max)
  cpu_baseline  the oracle (PyTorch-CPU IR-101 + reference-style per-probe
                search) on rank 0's host cores, on a bounded sample.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from facerecognitionpipeline_amd import weights as W  # noqa: E402
from facerecognitionpipeline_amd.arch import flop_per_face  # noqa: E402
from facerecognitionpipeline_amd.detector_arch import detector_macs  # noqa: E402

METRIC = "faces/sec embed+match (IR-101, 112×112, gallery=1k) at 1/2/4/8 GPU"
FP32_MFMA_PEAK_TFLOPS = 157.3
BF16_MFMA_PEAK_TFLOPS = 2500.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default 1, or WORLD_SIZE under torchrun): started here as child "
                         "processes unless torchrun already did")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only for tests)")
    ap.add_argument("--same-gpu", action="store_true",
                    help="testing: every rank on cuda:0 (needs --dist-backend gloo; RCCL refuses two ranks "
                         "on one GPU)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c3",
                    help="BASELINE.json config: c2 IR-50 embed-only B=256; c3 IR-101 embed+match B=256 G=1k "
                         "(default, the headline metric); c4 1080p frames -> SCRFD-10G detect -> align + "
                         "blur/quality gate + embed + match; c5 IR-101 embed+match B=256/GPU G=100k")
    ap.add_argument("--model-type", choices=["adaface", "arcface"], default="adaface",
                    help="embedding family (arcface = insightface IResNet weights, face_embedder.py:64-88)")
    ap.add_argument("--faces-per-frame", type=int, default=8, help="c4: faces per 1080p frame")
    ap.add_argument("--c4-pipeline", choices=["on", "off"], default="on",
                    help="c4: detect the next batch's frames on a second stream while this batch embeds + "
                         "matches (on), or run every stage back to back (off)")
    ap.add_argument("--arch", default=None)
    ap.add_argument("--batch", type=int, default=256, help="crops per GPU per step")
    ap.add_argument("--gallery", type=int, default=None, help="gallery rows (0 = embed only)")
    ap.add_argument("--topk", type=int, default=5)
    ap.add_argument("--precision", choices=["fp32", "bf16x3"], default="fp32",
                    help="conv arithmetic: exact f32 MFMA (default, parity path) or opt-in split bf16x3")
    ap.add_argument("--conv-algorithm", choices=["winograd4", "winograd", "direct"], default="winograd4",
                    help="stride-1 3x3 convs: Winograd F(4x4,3x3), F(2x2,3x3) or the direct implicit GEMM (all f32)")
    ap.add_argument("--lanes-min", type=int, default=None,
                    help="a forward of n >= 2x this many crops runs as two concurrent halves (0: one lane; default: library's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--exchange-reps", type=int, default=3,
                    help="N > 1: timed repeats of the gallery broadcast after the real one (steady-state rate)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per conv launch (tools/prof_summary.py --json); "
                         "default: the newest profiles/r*/layers_pmc.json")
    return ap.parse_args()


def host_cpu():
    """(threads to use, description) for the CPU baseline: one thread per PHYSICAL core this
    process may run on, bounded by the cgroup CPU quota when one is set."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    cores, model, machine_cores = set(), "unknown CPU", set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                core = f.read().strip()
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                pkg = f.read().strip()
            cores.add((pkg, core))
        except OSError:
            cores.add(("?", str(c)))
    try:
        with open("/proc/cpuinfo") as f:
            lines = f.read().splitlines()
        model = next(l.split(":", 1)[1].strip() for l in lines if l.startswith("model name"))
        phys = cid = None
        for l in lines:
            if l.startswith("physical id"):
                phys = l.split(":", 1)[1].strip()
            elif l.startswith("core id"):
                cid = l.split(":", 1)[1].strip()
                machine_cores.add((phys, cid))
    except (OSError, StopIteration):
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    threads = len(cores) if quota is None else min(len(cores), quota)
    desc = (f"{model}: {len(machine_cores) or '?'} physical cores in the machine, {len(cpus)} logical CPUs / "
            f"{len(cores)} physical cores in this process's affinity"
            + (f", cgroup quota {quota} CPUs" if quota is not None else ""))
    return max(1, threads), desc


def cpu_baseline(arch, sd, gallery_np, crops, budget_s):
    """Oracle (reference CPU path restated) on a bounded sample: batch-32 embed + per-probe search."""
    from oracle.adaface_net import load_oracle
    from oracle import reference_path as rp
    threads, cpu = host_cpu()
    torch.set_num_threads(threads)
    model = load_oracle(arch, sd)
    ids = [f"S{i}" for i in range(gallery_np.shape[0])]
    names = {s: s for s in ids}
    rp.extract_embeddings_batch(model, list(crops[:32]))  # warm-up batch
    done, t0 = 0, time.perf_counter()
    while done < len(crops):
        e = rp.extract_embeddings_batch(model, list(crops[done:done + 32]), batch_size=32)
        for q in e:
            if gallery_np.shape[0] == 0:
                break
            gal = np.vstack([gallery_np[i] for i in range(gallery_np.shape[0])])  # per-query vstack, as the reference
            rp.search(gal, ids, names, q, top_k=5)
        done += len(e)
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 3), "unit": "faces/s", "cores": threads, "kind": "port", "cpu": cpu,
            "sample": f"{done} crops of the bench workload ({arch}, batch 32"
                      + (f", G={gallery_np.shape[0]} per-probe vstack+sgemv+argsort search" if gallery_np.shape[0] else
                         ", embed only") + f"), {dt:.1f} s on {threads} host threads"}


def cpu_baseline_c4(sd, det_sd, gallery_np, frames, lms, per_frame, budget_s):
    """C4's own CPU counterpart on a bounded sample of the same frames: restated SCRFD-10G detect
    (letterbox + network + decode + NMS), per face similarity fit + fixed-point warpAffine + blur
    score (face_recognition.py:31-99), then batch embed + per-probe search of the frame's faces."""
    from oracle.adaface_net import load_oracle
    from oracle import align_ref as AR, reference_path as rp, scrfd as SR
    threads, cpu = host_cpu()
    torch.set_num_threads(threads)
    det = SR.load_oracle(det_sd)
    model = load_oracle("ir_101", sd)
    ids = [f"S{i}" for i in range(gallery_np.shape[0])]
    names = {s: s for s in ids}
    tmpl = AR.reference_template(112)

    def one_frame(f):
        img = frames[f]
        dets = SR.detect(det, img, 0.5)
        lm = lms[f][:per_frame].copy()
        for j, d in enumerate(dets[:per_frame]):
            lm[j] = d["landmarks"]
        faces = [AR.warp_affine_linear(img, AR.fit_similarity(lm[j], tmpl), 112) for j in range(per_frame)]
        for x in faces:
            AR.blur_score(x)
        for q in rp.extract_embeddings_batch(model, faces, batch_size=32):
            rp.search(np.vstack([gallery_np[i] for i in range(gallery_np.shape[0])]), ids, names, q, top_k=5)
        return len(faces)

    one_frame(0)  # warm-up
    done, n_fr, t0 = 0, 0, time.perf_counter()
    while n_fr < frames.shape[0] and time.perf_counter() - t0 < budget_s:
        done += one_frame(n_fr)
        n_fr += 1
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 3), "unit": "faces/s", "cores": threads, "kind": "port", "cpu": cpu,
            "sample": f"{n_fr} of the bench's 1080p frames x {per_frame} faces (SCRFD-10G detect, align, blur, "
                      f"IR-101 embed, G={gallery_np.shape[0]} per-probe search), {dt:.1f} s on {threads} host threads"}


def build_id_of(version: str):
    """The content hash at the end of fr_version() ("... build <id>"), or None."""
    return version.rsplit("build ", 1)[-1].strip() if version and "build " in version else None


def profile_figures(traffic_json, family, build, same_workload):
    """PMC figures of the dominant kernel family from the committed profile of this workload:
    (traffic bytes per launch, algorithmic bytes per launch, MFMA-busy fraction, source, note).
    PMC counters need rocprofv3 passes of their own, so they come from profiles/r*/layers_pmc.json
    (tools/gpu_profile.sh) -- and only when that profile was taken on THIS library build (its
    build_id equals the loaded library's fr_version() hash); otherwise None with the reason."""
    import glob
    tj = traffic_json
    if tj is None:
        cands = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "layers_pmc.json")))
        tj = cands[-1] if cands else None
    if not same_workload:
        return None, None, None, None, "no PMC profile of this workload (the committed one is C3 fp32 F(4x4))"
    if not tj or not os.path.exists(tj):
        return None, None, None, None, "no PMC profile found"
    with open(tj) as f:
        pj = json.load(f)
    rel = os.path.relpath(tj, REPO)
    want = build_id_of(build)
    if pj.get("build_id") is None or pj.get("build_id") != want:
        return None, None, None, None, (f"{rel} was collected on build {pj.get('build_id')}, the loaded library is "
                                        f"build {want}: its PMC figures are not attached")
    kj = pj.get("kernels", {}).get(family, {})
    traffic = kj.get("hbm_bytes_per_launch")
    src = (rel + f" (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, same workload, build {want})"
           if traffic is not None else None)
    return traffic, kj.get("alg_bytes_per_launch"), kj.get("mfma_busy_frac"), src, None


def detector_profile_figures(build):
    """PMC figures of the detector's F(4x4) launches from the committed detector profile
    (profiles/r*/c4_layers_pmc.json, tools/gpu_det_profile.sh -> tools/det_prof_summary.py), only
    when it was taken on this library build: (HBM bytes per launch, algorithmic bytes per launch,
    MFMA-busy fraction, source, note)."""
    import glob
    cands = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "c4_layers_pmc.json")))
    if not cands:
        return None, None, None, None, "no detector PMC profile found"
    with open(cands[-1]) as f:
        pj = json.load(f)
    rel = os.path.relpath(cands[-1], REPO)
    want = build_id_of(build)
    if pj.get("build_id") != want:
        return None, None, None, None, (f"{rel} was collected on build {pj.get('build_id')}, the loaded library is "
                                        f"build {want}: its PMC figures are not attached")
    fam = pj.get("families", {}).get("wino4_kernel", {})
    n = fam.get("layers") or 0
    if not n or "hbm_bytes" not in fam:
        return None, None, None, None, f"{rel} has no PMC figures for wino4_kernel"
    return (fam["hbm_bytes"] / n, fam["alg_bytes"] / n, fam.get("mfma_busy_frac"),
            rel + f" (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE of tools/det_time.py, build {want})", None)


def detector_roofline(detector, frames, det_stream, build, reps=5):
    """The detector's own roofline, measured live: `reps` fr_detect calls of the step's frames on the
    detector stream with nothing else queued, HIP events around them (detect_ms per call, D2H of the
    detections included) and the handle's per-launch event pairs (fr_profile_*) for the conv
    families.  achieved / frac count the products F(4x4) performs on the MFMA pipe (fp32 peak)."""
    dm = detector.model
    torch.cuda.synchronize()
    dm.profile_enable(True)
    dm.profile_read()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(det_stream):
        e0.record(det_stream)
        for _ in range(reps):
            dm.detect(frames, detector.det_thresh, detector.max_faces)
        e1.record(det_stream)
    e1.synchronize()
    prof = dm.profile_read()
    dm.profile_enable(False)
    detect_ms = e0.elapsed_time(e1) / reps
    w, d = prof["winograd"], prof["direct"]
    n_fr = int(frames.shape[0])
    alg = 2.0 * detector_macs() * n_fr
    ach = w["exec_flop"] / (w["ms"] * 1e-3) / 1e12 if w["ms"] else 0.0
    traffic, alg_bytes, busy, src, note = detector_profile_figures(build)
    out = {"bound": "mfma",
           "kernel": "wino4_kernel (detector instances: every stride-1 3x3 conv of SCRFD-10G, F(4x4,3x3) f32)",
           "achieved": round(ach, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
           "traffic": traffic, "traffic_from_profile": traffic is not None, "traffic_source": src,
           "traffic_note": note, "alg_bytes_per_launch": alg_bytes,
           "mfma_busy_frac_from_profile": round(busy, 4) if busy is not None else None,
           "launches_per_detect": w["launches"] // reps, "avg_launch_ms": round(w["ms"] / max(w["launches"], 1), 5),
           "flop_per_launch": w["exec_flop"] / max(w["launches"], 1),
           "alg_equiv_tflops": round(w["flop"] / (w["ms"] * 1e-3) / 1e12, 3) if w["ms"] else 0.0,
           "share_of_detect": round(w["ms"] / (detect_ms * reps), 4),
           "other_conv_kernel": {"kernel": "conv_mfma_kernel (stride-2 / 2x2 / 1x1 convs)",
                                 "tflops": round(d["flop"] / (d["ms"] * 1e-3) / 1e12, 3) if d["ms"] else 0.0,
                                 "frac": round(d["flop"] / (d["ms"] * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)
                                 if d["ms"] else 0.0,
                                 "launches_per_detect": d["launches"] // reps,
                                 "share_of_detect": round(d["ms"] / (detect_ms * reps), 4)},
           "frames_per_detect": n_fr, "detect_ms": round(detect_ms, 4),
           "alg_flop_per_detect": alg, "detect_alg_tflops": round(alg / (detect_ms * 1e-3) / 1e12, 3),
           "library_build": build,
           "note": ("standalone detects (nothing else queued) after the timed steps; alg_flop_per_detect is the "
                    "reference network's direct-conv count (unpadded channels, full 640x640 canvas), "
                    "detect_alg_tflops its rate over the whole detect (letterbox to NMS + D2H)")}
    return out


PRESETS = {"c2": ("ir_50", 0), "c3": ("ir_101", 1000), "c4": ("ir_101", 1000), "c5": ("ir_101", 100_000)}


def c4_inputs(n_faces, per_frame, dev, seed=7):
    """Synthetic 1080p frames (resident in HBM) with per_frame face landmark sets each."""
    from facerecognitionpipeline_amd.face_recognition import reference_template
    rng = np.random.default_rng(seed)
    n_frames = (n_faces + per_frame - 1) // per_frame
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    frames = torch.randint(0, 256, (n_frames, 1080, 1920, 3), dtype=torch.uint8, device=dev, generator=gen)
    t = reference_template(112).astype(np.float64)
    lms = []
    for f in range(n_frames):
        cur = []
        for j in range(per_frame):
            s = rng.uniform(1.2, 2.5)
            th = rng.uniform(-0.3, 0.3)
            R = s * np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
            c = np.array([rng.uniform(200, 1720), rng.uniform(200, 880)])
            cur.append((t - 56) @ R.T + c)
        lms.append(np.array(cur, dtype=np.float32))
    return frames, lms


def count_gpus():
    """GPUs this process may use, counted WITHOUT initialising HIP (the launcher must not touch the
    GPU before it starts the rank processes): the KFD topology's GPU nodes (gpu_id != 0) whose DRM
    render node is openable here (a container exposes a subset), else amdsmi; capped by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.  None if neither source
    works (the caller refuses to launch rather than fall back to a HIP-initialising count)."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = None
    if os.path.isdir(base):
        n = 0
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "gpu_id")) as f:
                    if int(f.read().strip() or 0) == 0:
                        continue  # a CPU node
                minor = None
                with open(os.path.join(base, node, "properties")) as f:
                    for line in f:
                        if line.startswith("drm_render_minor"):
                            minor = int(line.split()[1])
            except (OSError, ValueError, IndexError):
                continue
            if minor is not None and minor > 0 and not os.access(f"/dev/dri/renderD{minor}", os.R_OK | os.W_OK):
                continue
            n += 1
    else:
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            try:
                n = len(amdsmi.amdsmi_get_processor_handles())
            finally:
                amdsmi.amdsmi_shut_down()
        except Exception:  # noqa: BLE001 -- no library / no driver: the count is unknown
            n = None
    if n is None:
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def resolve_world(gpus, env) -> int:
    """Ranks this run has: WORLD_SIZE under torchrun (``--gpus``, when given, must agree), else
    ``--gpus`` (default 1).  Exits non-zero on a disagreement."""
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            sys.exit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}")
        return world
    return 1 if gpus is None else gpus


def launch_ranks(args) -> int:
    """``--gpus N`` without torchrun: start N fresh rank processes (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* in their environment, the same argv) and return the first non-zero exit code, else 0.

    Runs before anything here touches the GPU: ``count_gpus`` reads the KFD topology (or amdsmi),
    never HIP, and the children are started as new processes (never exec'd from this one).  Rank
    0's stdout is this process's stdout, so the one JSON line comes through.
    """
    import signal
    import socket
    import subprocess
    n = args.gpus
    if args.same_gpu and args.dist_backend != "gloo":
        sys.exit("bench.py: --same-gpu needs --dist-backend gloo (RCCL refuses two ranks on one GPU)")
    visible = count_gpus()
    if visible is None:
        sys.exit("bench.py: cannot count the visible GPUs (no KFD topology, no amdsmi); refusing to launch ranks")
    if args.same_gpu:
        if visible < 1:
            sys.exit("bench.py: --same-gpu needs one visible GPU, found none")
    elif n > visible:
        sys.exit(f"bench.py: --gpus {n} but only {visible} GPU(s) are visible; refusing to run fewer ranks")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # same process group as this launcher: a signal to the group (a driver's timeout) reaches the
        # ranks too, and SIGTERM / SIGINT to the launcher alone is forwarded below
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))

    def forward(signum, _frame):
        for q in procs:
            if q.poll() is None:
                q.send_signal(signum)
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    # a dead rank leaves the others blocked in a collective: end them
                    for q in pending:
                        q.terminate()
            time.sleep(0.05)
    except BaseException:
        for q in procs:
            if q.poll() is None:
                q.kill()
        for q in procs:
            q.wait()
        raise
    return rc


def main():
    args = parse()
    arch0, gal0 = PRESETS[args.config]
    args.arch = args.arch or arch0
    args.gallery = gal0 if args.gallery is None else args.gallery
    world = resolve_world(args.gpus, os.environ)
    if "WORLD_SIZE" not in os.environ and world > 1:
        args.gpus = world
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_gpu and args.dist_backend != "gloo":
        sys.exit("bench.py: --same-gpu needs --dist-backend gloo")
    if args.same_gpu:
        local = 0
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
    sd = W.synthetic_state_dict(args.arch, model_type=args.model_type)
    emb = FaceEmbedder(architecture=args.arch, model_type=args.model_type, state_dict=sd, device=dev, max_batch=args.batch,
                       precision=args.precision, conv_algorithm=args.conv_algorithm, lanes_min=args.lanes_min)

    # gallery: rank 0 embeds min(G, 1000) synthetic gallery crops on its GPU and grows them to G
    # rows as normalize(e + 0.0214 z); RCCL broadcast to the other ranks
    G = args.gallery
    G0 = min(max(G, 1), 1000)
    gal_crops = W.synthetic_crops(G0, W.CROP_SEED_GALLERY)
    gallery = None
    if rank == 0 and G > 0:
        gallery = emb.embed_tensor(torch.from_numpy(gal_crops).to(dev))
        if G > G0:
            gallery = torch.from_numpy(W.expand_gallery(gallery.cpu().numpy(), G)).to(dev)
    exchange = None
    if world > 1 and G > 0:
        from facerecognitionpipeline_amd.distributed import broadcast_gallery
        red_dev = dev if args.dist_backend == "nccl" else "cpu"

        def timed_broadcast(src_tensor):
            # every rank enters together (the barrier also brings up the communicator, so its setup
            # is not in the time); host clock around the collective + device syncs, max over ranks
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = broadcast_gallery(src_tensor, G, dev, src=0)
            torch.cuda.synchronize()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return out, t.item()

        gallery, t_first = timed_broadcast(gallery)
        reps = [timed_broadcast(gallery if rank == 0 else None)[1] for _ in range(max(0, args.exchange_reps))]
        nbytes = G * 512 * 4
        t_ss = float(np.median(reps)) if reps else t_first
        exchange = {"collective": "broadcast", "backend": "rccl" if args.dist_backend == "nccl" else "gloo",
                    "bytes": nbytes, "ms": round(t_first * 1e3, 3),
                    "ms_steady": round(t_ss * 1e3, 3), "reps": len(reps),
                    # bytes delivered to the N-1 receiving ranks per second, and per receiving rank
                    # (= per xGMI link for a fan-out from rank 0; a ring's bus bandwidth likewise)
                    "GBps_aggregate": round(nbytes * (world - 1) / t_ss / 1e9, 3),
                    "GBps_per_receiver": round(nbytes / t_ss / 1e9, 3)}
    if G > 0:
        emb.model.gallery_set(gallery)

    # probes resident in HBM: noisy copies of gallery crops (rank-dependent)
    probes_np = W.probe_crops(gal_crops, args.batch, seed=W.CROP_SEED_PROBE + rank)
    rgb = torch.from_numpy(probes_np).to(dev)
    k = args.topk
    idx = torch.empty((args.batch, k), dtype=torch.int32, device=dev)
    score = torch.empty((args.batch, k), dtype=torch.float32, device=dev)
    e_out = torch.empty((args.batch, 512), dtype=torch.float32, device=dev)

    det_stats = {"detected": 0, "padded": 0}
    if args.config == "c4":
        from facerecognitionpipeline_amd.face_recognition import FaceDetector
        frames, lms = c4_inputs(args.batch, args.faces_per_frame, dev)
        # two crop buffers: batch i's align + blur run on their own stream (aux) into one while batch
        # i - 1's embed + match still read the other, so the blur's sync waits for this batch's
        # aligns only, and the embed of batch i is queued before batch i - 1's has finished
        crop_bufs = [torch.empty((args.batch, 112, 112, 3), dtype=torch.uint8, device=dev) for _ in range(2)]
        aux = torch.cuda.Stream(device=dev)
        embed_done = [None, None]  # event after the last embed + match that read each buffer
        step_no = [0]
        from facerecognitionpipeline_amd.detector_arch import synthetic_detector_state_dict
        detector_sd = synthetic_detector_state_dict()
        detector = FaceDetector(device=dev, max_frames=min(32, frames.shape[0]), max_faces=64, state_dict=detector_sd)
        # pipelined serving: batch i+1's detection is started (on its own non-blocking stream, from
        # a worker thread: fr_detect returns host detections and waits for its own stream) at the
        # start of step i, before batch i's align / gate / embed + match are queued on the main
        # stream, so the GPU always has the other workload queued while the host fits landmarks
        # or waits for a sync.  Every step still detects exactly one batch of frames inside the
        # timed region (the first batch's in warmup; the last step starts one detection that no
        # timed step consumes, so the timed region holds K detections either way).
        det_stream = torch.cuda.Stream(device=dev)
        pending = []
        det_pool = None
        if args.c4_pipeline == "on":
            from concurrent.futures import ThreadPoolExecutor
            det_pool = ThreadPoolExecutor(1, thread_name_prefix="c4-detect")

    def detect_job():
        with torch.cuda.stream(det_stream):
            return detector.model.detect(frames, detector.det_thresh, detector.max_faces)

    def detect_batch():
        if args.c4_pipeline == "on":
            return det_pool.submit(detect_job)
        return detector.model.detect(frames, detector.det_thresh, detector.max_faces)

    def step():
        if args.config == "c4":
            # SCRFD on every frame (batched); each frame's top faces_per_frame detections are aligned
            # (a frame with fewer is topped up with the synthetic placements so every step embeds
            # exactly `batch` faces); blur + gate on all crops; one embed+match
            got = pending.pop() if pending else detect_batch()
            dets, counts = got.result() if args.c4_pipeline == "on" else got
            if args.c4_pipeline == "on":
                pending.append(detect_batch())  # the next batch's detection, queued first
            b = step_no[0] % 2
            step_no[0] += 1
            crops = crop_bufs[b]
            with torch.cuda.stream(aux):
                if embed_done[b] is not None:
                    aux.wait_event(embed_done[b])  # the embed that last read this buffer
                o = 0
                for f in range(frames.shape[0]):
                    nf = min(args.faces_per_frame, args.batch - o)
                    nd = min(int(counts[f]), nf)
                    lm = lms[f][:nf].copy()
                    lm[:nd] = dets[f, :nd, 5:15].reshape(nd, 5, 2)
                    det_stats["detected"] += nd
                    det_stats["padded"] += nf - nd
                    emb.model.align_faces(frames[f], lm, 112, crops[o:o + nf])
                    o += nf
                # syncs the aux stream only: this batch's aligns + blur
                blur = emb.model.blur_scores(crops)
            if not (blur >= 0).all():
                raise RuntimeError("bad blur scores")
            main = torch.cuda.current_stream(dev)
            main.wait_stream(aux)
            emb.model.embed_match(crops, k, idx, score, e_out)
            embed_done[b] = main.record_event()
        elif G > 0:
            emb.model.embed_match(rgb, k, idx, score, e_out)
        else:
            emb.model.embed(rgb, e_out, True)

    for _ in range(args.warmup):
        step()

    def timed_steps():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        tmin = t.clone()
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.all_reduce(tmin, op=dist.ReduceOp.MIN)
        rank_spread[:] = [tmin.item(), t.item()]
        return t.item()

    # throughput: the K steps with nothing else on the queue; then the same K steps again with a
    # HIP event pair around every launch (fr_profile_*) for the per-kernel roofline -- the event
    # records add ~0.8 ms per IR-101 step, so they stay out of the throughput pass
    rank_spread = [0.0, 0.0]
    tmax = timed_steps()
    rank_ms = [round(x / args.steps * 1e3, 3) for x in rank_spread]
    emb.model.profile_enable(True)
    emb.model.profile_read()
    tprof = timed_steps()
    prof = emb.model.profile_read()
    emb.model.profile_enable(False)
    if args.config == "c4" and det_pool is not None:
        for f in pending:  # the detection the last step started (no timed step consumes it)
            f.result()
        pending.clear()
        det_pool.shutdown()

    # sanity: probes are noisy copies of gallery rows i % G
    top1_ok = (float((idx[:, 0].cpu().numpy() == np.arange(args.batch) % G0).mean())
               if G > 0 and args.config != "c4" else None)
    if world > 1 and top1_ok is not None:
        # the worst rank's self-match rate (every rank's probes are noisy copies of rows i % G0)
        t1 = torch.tensor([top1_ok], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t1, op=dist.ReduceOp.MIN)
        top1_ok = t1.item()

    if rank == 0:
        faces = world * args.batch * args.steps
        # dominant kernel = the conv family with the most time in the timed region (HIP events on the
        # launch stream): the Winograd kernel for the f32 default, the direct implicit-GEMM one otherwise
        fams = {f: prof[f] for f in ("winograd", "direct") if prof[f]["launches"]}
        dom = max(fams, key=lambda f: fams[f]["ms"])
        kp = fams[dom]
        alg_tflops = kp["flop"] / (kp["ms"] * 1e-3) / 1e12
        exec_tflops = kp["exec_flop"] / (kp["ms"] * 1e-3) / 1e12
        conv_tflops = prof["conv_flop"] / (prof["conv_ms"] * 1e-3) / 1e12 if prof["conv_ms"] > 0 else 0.0
        # bf16x3 executes 3 bf16 MFMA products per algorithmic f32 product: its executed fraction is
        # taken against the dense bf16 MFMA peak
        peak, mult = (FP32_MFMA_PEAK_TFLOPS, 1.0) if args.precision == "fp32" else (BF16_MFMA_PEAK_TFLOPS, 3.0)
        from facerecognitionpipeline_amd import _lib as frlib
        build = frlib.load().fr_version().decode()
        same_workload = (args.config == "c3" and args.model_type == "adaface" and args.arch == "ir_101"
                         and args.batch == 256 and G == 1000 and args.precision == "fp32"
                         and args.conv_algorithm == "winograd4")
        traffic, alg_bytes, mfma_busy, traffic_src, traffic_note = profile_figures(
            args.traffic_json, dom, build, same_workload)
        if args.conv_algorithm != "winograd4":
            wino_name = "wino_kernel (Winograd F(2x2,3x3) f32, every stride-1 3x3 conv)"
        else:
            wino_name = ("wino4_kernel (Winograd F(4x4,3x3) f32: fused input transform, 16x16x4 MFMA, lane-local "
                         "output transform; every stride-1 3x3 conv)")
        kernel_name = {"winograd": wino_name,
                       "direct": "conv_mfma_kernel (implicit-GEMM; every conv/FC launch in this mode)"}[dom]
        # achieved = the FLOPs the kernel's algorithm performs per launch / its average launch time:
        # direct conv 2*M*N*K; Winograd F(m x m, 3x3) 2 * (m+2)^2 products per m x m output tile
        # (canvas tiles) and (cin, cout) pair -- the work on the MFMA pipe, so frac <= 1 is the MFMA
        # utilisation.  alg_equiv_tflops is the direct-conv-equivalent rate of the same launches.
        ach = exec_tflops if dom == "winograd" else alg_tflops
        roofline = {"bound": "mfma", "kernel": kernel_name,
                    "achieved": round(ach, 3), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(ach * mult / peak, 4),
                    # traffic is NOT observed in this run: PMC counters need their own rocprofv3 passes,
                    # so it is read from the committed profile of the same workload (traffic_source)
                    "traffic": traffic, "traffic_from_profile": traffic is not None,
                    "traffic_source": traffic_src, "traffic_note": traffic_note, "library_build": build,
                    "alg_bytes_per_launch": alg_bytes,
                    # PMC SQ_VALU_MFMA_BUSY_CYCLES / (1,024 SIMDs x GRBM_GUI_ACTIVE / 8) of the same kernel in
                    # the committed profile of this workload (its own rocprofv3 pass, like traffic)
                    "mfma_busy_frac_from_profile": round(mfma_busy, 4) if mfma_busy is not None else None,
                    "launches": kp["launches"],
                    "flop_per_launch": (kp["exec_flop"] if dom == "winograd" else kp["flop"]) / kp["launches"],
                    "avg_launch_ms": round(kp["ms"] / kp["launches"], 5),
                    "share_of_step": round(kp["ms"] / max(prof["total_ms"], 1e-9), 4)}
        if dom == "winograd":
            roofline["alg_equiv_tflops"] = round(alg_tflops, 3)
            roofline["note"] = ("achieved/frac count the products Winograd performs on the MFMA pipe ("
                                + ("36 per 4x4 canvas tile" if args.conv_algorithm == "winograd4" else "16 per 2x2 tile")
                                + " and cin x cout pair); alg_equiv_tflops counts direct-conv FLOPs (2*M*N*K), "
                                  "which Winograd needs " + ("4x" if args.conv_algorithm == "winograd4" else "2.25x")
                                + " fewer of, so it can exceed the peak")
        if "direct" in fams and dom != "direct":
            d = fams["direct"]
            roofline["other_conv_kernel"] = {"kernel": "conv_mfma_kernel (stride-2 / 1x1 convs, FC, gallery scores)",
                                             "tflops": round(d["flop"] / (d["ms"] * 1e-3) / 1e12, 3),
                                             "frac": round(d["flop"] / (d["ms"] * 1e-3) / 1e12 / peak, 4),
                                             "launches": d["launches"],
                                             "share_of_step": round(d["ms"] / max(prof["total_ms"], 1e-9), 4)}
        roofline["conv_family_tflops"] = round(conv_tflops, 3)
        out = {
            "metric": METRIC if args.config == "c3" and args.model_type == "adaface" else (
                f"faces/sec detect+align+quality+embed+match from 1080p frames (IR-101, gallery={G})"
                if args.config == "c4" else
                f"faces/sec embed-only ({args.arch.upper().replace('_', '-')}, 112×112)" if G == 0 else
                f"faces/sec embed+match ({args.arch.upper().replace('_', '-')}, 112×112, gallery={G})"),
            "value": round(faces / tmax, 2),
            "unit": "faces/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1e3, 3),
            "ms_per_step_profiled_pass": round(tprof / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.precision == "fp32" else "bf16x3 (f32 operands split hi+lo, f32 accumulate)",
            "data": ("synthetic (seeded random 1080p uint8 frames; seeded random-init SCRFD-10G and AdaFace "
                     "weights; frames with fewer detections than faces-per-frame are topped up with seeded "
                     "5-point placements)" if args.config == "c4" else
                     "synthetic (seeded uint8 crops; seeded random-init AdaFace weights)"),
            "config": {"workload": (f"{args.config.upper()}: "
                                    + (f"1080p frames ({args.faces_per_frame} faces each) -> SCRFD-10G detect "
                                       "(640x640 letterbox) -> device align + blur/quality gate + "
                                       if args.config == "c4" else "")
                                    + f"{args.arch.upper().replace('_', '-')} "
                                    + ("AdaFace" if args.model_type == "adaface" else "ArcFace (IResNet)") + " embed"
                                    + (f" + cosine top-{k} match vs {G}-row gallery" if G > 0 else " only")
                                    + f", batch {args.batch}/GPU, 112x112 uint8 RGB"),
                       "arch": args.arch, "batch_per_gpu": args.batch, "global_batch": args.batch * world,
                       "gallery": G, "top_k": k, "parallelism": f"dp{world}",
                       "gallery_exchange": (("rccl broadcast" if args.dist_backend == "nccl" else "gloo broadcast")
                                            if world > 1 else "none"),
                       **({"ranks_share_gpu": True} if args.same_gpu and world > 1 else {}),
                       # concurrent half-batch forwards per GPU (fr_set_lanes; library default 64 crops
                       # per lane, at most 2 lanes); the roofline pass always runs one lane
                       "lanes": (1 if args.lanes_min == 0 else
                                 max(1, min(2, args.batch // (64 if args.lanes_min is None else args.lanes_min)))),
                       **({"frames_per_step": int(frames.shape[0]),
                           "detect_overlaps_embed": args.c4_pipeline == "on",
                           "detector_gflop_per_frame": round(2 * detector_macs() / 1e9, 3),
                           "aligned_from_detections": det_stats["detected"],
                           "aligned_from_padding": det_stats["padded"]} if args.config == "c4" else {})},
            "flop_per_face": flop_per_face(args.arch, G, args.model_type),
            "path_tflops": round(faces / tmax * flop_per_face(args.arch, G, args.model_type) / 1e12, 2),
            "top1_self_match": top1_ok,
            "roofline": roofline,
        }
        if args.config == "c4":
            roofline["detector"] = detector_roofline(detector, frames, det_stream, build)
        if world > 1:
            # the fastest and the slowest rank's timed region (value uses the slowest)
            out["rank_ms_per_step_min"], out["rank_ms_per_step_max"] = rank_ms
            # the path's only collective, outside the timed region: the G x 512 gallery broadcast
            out["gallery_exchange"] = exchange
            if exchange is not None:
                out["gallery_exchange_ms"] = exchange["ms"]
                out["gallery_exchange_GBps"] = exchange["GBps_aggregate"]
        if world == 1 and not args.no_cpu_baseline and args.model_type == "adaface":
            gnp = gallery.cpu().numpy() if G > 0 else np.zeros((0, 512), np.float32)
            if args.config == "c4":
                out["cpu_baseline"] = cpu_baseline_c4(sd, detector_sd, gnp, frames.cpu().numpy(), lms,
                                                      args.faces_per_frame, args.cpu_seconds)
            else:
                sample = W.probe_crops(gal_crops, 1024, seed=W.CROP_SEED_PROBE)
                out["cpu_baseline"] = cpu_baseline(args.arch, sd, gnp, sample, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
