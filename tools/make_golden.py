#!/usr/bin/env python3
"""Generate tests/golden/* by running the REFERENCE code in the build container.

Runs only where ``/root/reference`` exists (never on the GPU box).  It imports
the reference's own ``face_embedder.FaceEmbedder`` and
``gallery_manager.GalleryManager`` and records their outputs on seeded inputs:

* ``embed_<arch>.npz`` — reference ``extract_embeddings_batch`` (batch 32,
  face_embedder.py:137-182) on seeded gallery crops, reference
  ``extract_embedding`` (face_embedder.py:112-135) on seeded probe crops, and
  reference ``GalleryManager.search(top_k=5)`` (gallery_manager.py:189-205)
  for every probe against a gallery built with ``add_student``.
* ``c3_ir_101.npz`` — the headline configuration exactly (BASELINE.json
  configs[2]): reference IR-101 ``extract_embeddings_batch`` of the bench's
  1,000 gallery crops and 256 probe crops, a 1,000-row gallery built with the
  reference ``GalleryManager.add_student``, and reference ``search(top_k=5)``
  of every probe (gallery_manager.py:189-205).
* ``resize_ir_50.npz`` — reference ``extract_embeddings_batch`` on crops that
  are not 112x112 (224x224 enrollment crops, enroll_students.py:67-81,222, and
  odd sizes), i.e. through the ``cv2.resize`` branch of face_embedder.py:94-96.
  cv2 is absent, so for this file the stub's ``resize`` is the restatement of
  OpenCV's INTER_LINEAR in ``oracle/scrfd.py``: the fixture pins the
  reference wrapper's order of operations around it, not cv2 itself.
* ``backup_<name>.npz`` — the reference's committed gallery backups
  (``gallery/backups/*.json`` and ``backups/*.json``, export format
  gallery_manager.py:246-270) as arrays, plus reference ``GalleryManager``
  templates rebuilt by ``add_student`` and reference ``search`` results for
  every stored sample.  ``backups/adaface_ir_50_backup_20251202_081742.json``
  becomes ``backup_root_adaface_ir_50.npz``.
* ``gate.npz`` — the reference ``FaceQualityFilter.compute_pose_angles`` /
  ``is_valid`` and ``FaceProcessor.process_numpy`` (face_recognition.py:101-216)
  on the seeded frame and fixed detections of ``tests/_gate_inputs.py``, for
  three quality configurations, RGB and grayscale frames, ``return_all``
  true and false: every result's detection index, ``is_valid``, metrics
  (values and types) and aligned-crop SHA-256.  ``insightface`` is absent and
  is stubbed (``FaceAnalysis`` refuses to be built; the processor gets a
  fixed-detection detector); the cv2 calls go to the restatements in
  ``oracle/align_ref.py``, so this file pins the reference's gate logic,
  pose arithmetic, ordering and dict layout -- everything but cv2's own
  numerics.
* ``image.npz`` + ``image_{rgb,gray,rgba}.png`` — small seeded PNG files (RGB, 8-bit
  gray, RGBA) and the SHA-256 of the RGB array ``cv2.imread`` + ``COLOR_BGR2RGB`` yields
  for each (gray expanded to 3 channels, alpha dropped: IMREAD_COLOR), computed from the
  arrays the files were written from; and the reference ``FaceProcessor.process_image``
  (face_recognition.py:174-182) on the gate frame written as PNG (``imread`` in the cv2
  shim decodes through PIL: lossless, so the pixels are the frame's), with the gate's
  fixed detections, default quality settings, ``return_all`` true and false.
* ``dropin_students.pkl`` + ``dropin_students.npz`` — a gallery written by THIS repo's
  ``GalleryManager.save`` (``ref_students.pkl`` loaded, one student enrolled, one updated,
  one deleted through the drop-in), then loaded by the REFERENCE ``GalleryManager`` (the real
  ``pickle.load`` of gallery_manager.py:241-242): the records it sees (ids, names, sample
  counts, dates, array checksums) and its ``search(top_k=5)`` of every stored sample.
* ``ref_students.pkl`` / ``ref_students.json`` — the reference's own gallery
  FILES (gallery_manager.py:207-232): a reference ``GalleryManager`` built
  with ``add_student`` (samples + metadata) from
  ``gallery/backups/adaface_ir_101_backup_*.json`` and ``.save()``d.  Its
  templates and search results are those of ``backup_adaface_ir_101.npz``.

Two modules the reference imports are absent from this image and are supplied
in a temporary directory that is put on ``sys.path`` for this run only:
``net`` (upstream AdaFace, restated in ``oracle/adaface_net.py``) and ``cv2``
(only ``cv2.resize``/``INTER_LINEAR`` are referenced on the embed path; the
stub raises unless the resize restatement is switched on for the resize
fixture).  Weights are the seeded synthetic checkpoint of
``facerecognitionpipeline_amd.weights`` saved in the reference's checkpoint
format.  Crops are regenerated from their seeds at test time; their SHA-256 is
stored to pin them.

Usage: ``python tools/make_golden.py [embed] [c3] [resize] [backups] [refpkl] [gate] [image] [dropin]``
(no argument: all).
"""
from __future__ import annotations

import contextlib
import glob
import hashlib
import io
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from facerecognitionpipeline_amd import weights as W  # noqa: E402

N_GALLERY = 8
N_PROBE = 8
TOP_K = 5

C3_GALLERY = 1000   # BASELINE.json configs[2]: gallery=1k, batch=256, top-5
C3_PROBES = 256
RESIZE_SIZES = ((224, 224),) * 6 + ((150, 130), (96, 96))   # (H, W) of the resize-branch crops
RESIZE_SEED = 0xFACE0224

CV2_STUB = '''import sys
INTER_LINEAR = 1
RESTATED_RESIZE = False
def resize(img, dsize, interpolation=INTER_LINEAR):
    if not RESTATED_RESIZE:
        raise RuntimeError("cv2 stub: resize is not expected on the 112x112 golden path")
    sys.path.insert(0, {repo!r})
    from oracle.scrfd import resize_linear_u8  # restatement of cv::resize INTER_LINEAR (uint8)
    assert interpolation == INTER_LINEAR
    return resize_linear_u8(img, int(dsize[0]), int(dsize[1]))

# face_recognition.py's calls (gate fixture): delegated to the restatements in oracle/align_ref.py
COLOR_RGB2BGR = COLOR_BGR2RGB = 4
COLOR_RGB2GRAY = 7
COLOR_GRAY2BGR = 8
CV_64F = 6
BORDER_CONSTANT = 0
def _A():
    sys.path.insert(0, {repo!r})
    from oracle import align_ref
    return align_ref
def cvtColor(img, code):
    import numpy as np
    if code == COLOR_RGB2BGR:
        return np.ascontiguousarray(img[..., ::-1])
    if code == COLOR_GRAY2BGR:
        return np.repeat(img[..., None], 3, axis=2)
    if code == COLOR_RGB2GRAY:
        return _A().rgb_to_gray(img)
    raise NotImplementedError(code)
def estimateAffinePartial2D(src, dst):
    return _A().fit_similarity(src, dst), None
def getAffineTransform(src, dst):
    raise NotImplementedError("not on the similarity path")
def warpAffine(img, M, dsize, flags=INTER_LINEAR, borderMode=BORDER_CONSTANT, borderValue=0):
    assert flags == INTER_LINEAR and borderMode == BORDER_CONSTANT and borderValue == 0 and dsize[0] == dsize[1]
    if img.ndim == 2:
        return _A().warp_affine_linear(img[:, :, None], M, int(dsize[0]))[:, :, 0]
    return _A().warp_affine_linear(img, M, int(dsize[0]))
def imread(path, flags=1):
    # IMREAD_COLOR of an 8-bit file: 3-channel BGR, or None when unreadable; decoded by PIL
    # (lossless formats decode to the same bytes; this pins process_image's wrapper, not imread)
    import numpy as np
    try:
        from PIL import Image
        with Image.open(path) as im:
            im.load()
            return np.ascontiguousarray(np.asarray(im.convert("RGB"), dtype=np.uint8)[..., ::-1])
    except (OSError, ValueError, SyntaxError):
        return None
def Laplacian(gray, ddepth):
    import numpy as np
    assert ddepth == CV_64F
    g = gray.astype(np.float64)
    p = np.pad(g, 1, mode="reflect")  # BORDER_REFLECT_101, ksize 1: [0 1 0; 1 -4 1; 0 1 0]
    return p[:-2, 1:-1] + p[2:, 1:-1] + p[1:-1, :-2] + p[1:-1, 2:] - 4.0 * g
'''
# insightface is absent: FaceAnalysis('buffalo_l') would download its model pack, so the stub
# refuses to be constructed; FaceProcessor gets a fixed-detection stub detector instead
INSIGHTFACE_APP = '''class FaceAnalysis:
    def __init__(self, *a, **k):
        raise RuntimeError("insightface stub: FaceAnalysis is never constructed for the golden files")
'''
NET_SHIM = '''import sys
sys.path.insert(0, {repo!r})
from oracle.adaface_net import build_model  # restated upstream AdaFace net.py
'''


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def quiet():
    return contextlib.redirect_stdout(io.StringIO())


def main() -> None:
    if not os.path.isdir(REF):
        raise SystemExit("reference not present; golden files are generated in the build container only")
    parts = set(sys.argv[1:]) or {"embed", "c3", "resize", "backups", "refpkl", "gate", "image", "dropin"}
    os.makedirs(OUT, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="frgolden_")
    with open(os.path.join(tmp, "cv2.py"), "w") as f:
        f.write(CV2_STUB.format(repo=REPO))
    with open(os.path.join(tmp, "net.py"), "w") as f:
        f.write(NET_SHIM.format(repo=REPO))
    for d in ("insightface", os.path.join("insightface", "utils")):
        os.makedirs(os.path.join(tmp, d), exist_ok=True)
        open(os.path.join(tmp, d, "__init__.py"), "w").close()
    with open(os.path.join(tmp, "insightface", "app.py"), "w") as f:
        f.write(INSIGHTFACE_APP)
    open(os.path.join(tmp, "insightface", "utils", "face_align.py"), "w").close()
    sys.path.insert(0, tmp)
    sys.path.append(REF)
    import torch
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    import face_embedder as ref_fe  # reference module
    import gallery_manager as ref_gm  # reference module

    def embedder(arch):
        ckpt = os.path.join(tmp, f"{arch}.ckpt")
        if not os.path.exists(ckpt):
            W.save_checkpoint(W.synthetic_state_dict(arch), ckpt)
        with quiet():
            return ref_fe.FaceEmbedder(architecture=arch, model_path=ckpt, model_type="adaface",
                                       device=torch.device("cpu"))

    def search_arrays(gm, queries):
        with quiet():
            res = [gm.search(q, top_k=TOP_K) for q in queries]
            gal, ids = gm.get_gallery_embeddings()
        pos = {sid: i for i, sid in enumerate(ids)}
        idx = np.array([[pos[sid] for sid, _n, _s in r] for r in res], dtype=np.int32)
        sc = np.array([[s for _sid, _n, s in r] for r in res], dtype=np.float32)
        return gal, idx, sc

    if "embed" in parts:
        base = W.synthetic_crops(N_GALLERY, W.CROP_SEED_GALLERY)
        probes = W.probe_crops(base, N_PROBE)
        for arch in ("ir_50", "ir_101"):
            emb = embedder(arch)
            with quiet():
                g = emb.extract_embeddings_batch(list(base), normalize=True, batch_size=32)
                p = np.stack([emb.extract_embedding(x, normalize=True) for x in probes])
                gm = ref_gm.GalleryManager(gallery_path=os.path.join(tmp, f"g_{arch}", "students.pkl"))
                for i in range(N_GALLERY):
                    gm.add_student(f"S{i:03d}", f"N{i}", g[i])
            gal, ids_arr, sc_arr = search_arrays(gm, p)
            np.savez_compressed(
                os.path.join(OUT, f"embed_{arch}.npz"),
                weight_seed=np.int64(W.DEFAULT_WEIGHT_SEED), gallery_seed=np.int64(W.CROP_SEED_GALLERY),
                probe_seed=np.int64(W.CROP_SEED_PROBE),
                gallery_crops_sha256=np.array(sha(base)), probe_crops_sha256=np.array(sha(probes)),
                gallery_emb=g.astype(np.float32), probe_emb=p.astype(np.float32),
                gallery_matrix=gal.astype(np.float32),
                search_idx=ids_arr, search_score=sc_arr)
            print(arch, "gallery", g.shape, "probe", p.shape, "top1", ids_arr[:, 0].tolist())

    if "c3" in parts:
        # exactly the bench workload (bench.py: W.synthetic_crops(1000, CROP_SEED_GALLERY) and rank 0's
        # W.probe_crops(gal, 256, seed=CROP_SEED_PROBE)); every probe through the reference embedder,
        # every gallery row through add_student, every search through the reference search
        gal_crops = W.synthetic_crops(C3_GALLERY, W.CROP_SEED_GALLERY)
        probes = W.probe_crops(gal_crops, C3_PROBES, seed=W.CROP_SEED_PROBE)
        emb = embedder("ir_101")
        with quiet():
            g = emb.extract_embeddings_batch(list(gal_crops), normalize=True, batch_size=32)
            p = emb.extract_embeddings_batch(list(probes), normalize=True, batch_size=32)
            gm = ref_gm.GalleryManager(gallery_path=os.path.join(tmp, "c3", "students.pkl"))
            for i in range(C3_GALLERY):
                gm.add_student(f"S{i:04d}", f"N{i}", g[i])
        gal, ids_arr, sc_arr = search_arrays(gm, p)
        # single-sample add_student keeps the row as is (gallery_manager.py:298-299): the reference
        # gallery matrix IS the embedding matrix, stored once
        assert np.array_equal(gal, g)
        np.savez_compressed(
            os.path.join(OUT, "c3_ir_101.npz"),
            weight_seed=np.int64(W.DEFAULT_WEIGHT_SEED), gallery_seed=np.int64(W.CROP_SEED_GALLERY),
            probe_seed=np.int64(W.CROP_SEED_PROBE),
            gallery_crops_sha256=np.array(sha(gal_crops)), probe_crops_sha256=np.array(sha(probes)),
            gallery_emb=g.astype(np.float32), probe_emb=p.astype(np.float32),
            search_idx=ids_arr, search_score=sc_arr)
        print("c3", g.shape, p.shape, "top1 == i mod G:", float((ids_arr[:, 0] == np.arange(C3_PROBES) % C3_GALLERY).mean()))

    if "resize" in parts:
        import cv2  # the stub above
        cv2.RESTATED_RESIZE = True
        r = np.random.Generator(np.random.PCG64(RESIZE_SEED))
        crops = [r.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for h, w in RESIZE_SIZES]
        emb = embedder("ir_50")
        with quiet():
            e = emb.extract_embeddings_batch(crops, normalize=True, batch_size=32)
        cv2.RESTATED_RESIZE = False
        np.savez_compressed(
            os.path.join(OUT, "resize_ir_50.npz"), weight_seed=np.int64(W.DEFAULT_WEIGHT_SEED),
            crop_seed=np.int64(RESIZE_SEED), sizes=np.array(RESIZE_SIZES, dtype=np.int32),
            crops_sha256=np.array(sha(np.concatenate([c.ravel() for c in crops]))), emb=e.astype(np.float32))
        print("resize", e.shape)

    if "backups" in parts:
        paths = sorted(glob.glob(os.path.join(REF, "gallery", "backups", "*.json")))
        paths += sorted(glob.glob(os.path.join(REF, "backups", "*.json")))
        for path in paths:
            name = os.path.basename(path).split("_backup_")[0]
            if os.path.dirname(path) == os.path.join(REF, "backups"):
                name = "root_" + name
            with open(path) as f:
                data = json.load(f)
            sids = list(data["students"].keys())
            emb = np.array([data["students"][s]["embeddings"] for s in sids], dtype=np.float32)
            tmpl = np.array([data["students"][s]["template_embedding"] for s in sids], dtype=np.float32)
            avg = np.array([data["students"][s]["metadata"].get("avg_similarity", np.nan) for s in sids],
                           dtype=np.float64)
            with quiet():
                gm = ref_gm.GalleryManager(gallery_path=os.path.join(tmp, f"b_{name}", "students.pkl"),
                                           aggregation_method="mean")
                for s in sids:
                    gm.add_student(s, data["students"][s]["name"], np.array(data["students"][s]["embeddings"],
                                                                             dtype=np.float32))
            gal, idx, sc = search_arrays(gm, emb.reshape(-1, emb.shape[-1]))
            np.savez_compressed(
                os.path.join(OUT, f"backup_{name}.npz"),
                student_ids=np.array(sids), embeddings=emb, stored_template=tmpl, avg_similarity=avg,
                ref_template=gal.astype(np.float32), search_idx=idx, search_score=sc)
            print(name, emb.shape)

    if "refpkl" in parts:
        import shutil
        path = sorted(glob.glob(os.path.join(REF, "gallery", "backups", "adaface_ir_101_backup_*.json")))[0]
        with open(path) as f:
            data = json.load(f)
        d = os.path.join(tmp, "refpkl")
        with quiet():
            gm = ref_gm.GalleryManager(gallery_path=os.path.join(d, "students.pkl"), aggregation_method="mean")
            for sid, rec in data["students"].items():
                gm.add_student(sid, rec["name"], np.array(rec["embeddings"], dtype=np.float32),
                               metadata=rec.get("metadata") or {})
            gm.save()
        shutil.copyfile(os.path.join(d, "students.pkl"), os.path.join(OUT, "ref_students.pkl"))
        shutil.copyfile(os.path.join(d, "students.json"), os.path.join(OUT, "ref_students.json"))
        print("refpkl", len(data["students"]), "students from", os.path.basename(path))

    if "gate" in parts:
        import face_recognition as ref_fr  # reference module (insightface / cv2 stubbed above)
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import _gate_inputs as GI
        frame = GI.frame()
        dets = GI.detections()

        class FixedDetector:  # the reference detector's output contract (face_recognition.py:37-48)
            def detect(self, image):
                return [{"bbox": d["bbox"].copy(), "landmarks": d["landmarks"].copy(), "det_score": d["det_score"],
                         "pose": None, "age": None, "gender": None} for d in dets]

        def enc(v):
            return {"v": float(v), "t": type(v).__name__}

        records = []
        for ci, cfg in enumerate(GI.QUALITY_CONFIGS):
            qf = ref_fr.FaceQualityFilter(**cfg)
            al = ref_fr.FaceAligner(output_size=GI.S)
            fp = ref_fr.FaceProcessor.__new__(ref_fr.FaceProcessor)  # __init__ would build FaceAnalysis
            fp.detector, fp.aligner, fp.quality_filter = FixedDetector(), al, qf
            for kind, img in (("rgb", frame), ("gray", GI.frame_gray(frame))):
                with quiet():
                    per_face = []
                    for d in dets:
                        crop = al.align(img, d["landmarks"])
                        ok, m = qf.is_valid(d, crop)
                        per_face.append({"is_valid": bool(ok), "metrics": {k: enc(v) for k, v in m.items()},
                                         "pose": {k: enc(v) for k, v in qf.compute_pose_angles(d["landmarks"]).items()},
                                         "crop_sha256": sha(crop)})
                    runs = {}
                    for ra in (False, True):
                        res = fp.process_numpy(img, return_all=ra)
                        runs[str(ra)] = [{"det": next(i for i, d in enumerate(dets)
                                                      if np.array_equal(d["landmarks"], r["landmarks"])),
                                          "is_valid": bool(r["is_valid"]), "det_score": r["det_score"],
                                          "metrics": {k: enc(v) for k, v in r["quality_metrics"].items()},
                                          "crop_sha256": sha(r["aligned_face"]), "crop_ndim": int(r["aligned_face"].ndim),
                                          "keys": sorted(r)} for r in res]
                records.append({"config": ci, "frame": kind, "per_face": per_face, "process_numpy": runs})
        np.savez_compressed(os.path.join(OUT, "gate.npz"), frame_sha256=np.array(sha(frame)),
                            records=np.array(json.dumps(records)))
        valid = sum(f["is_valid"] for r in records for f in r["per_face"])
        print("gate", len(records), "runs,", valid, "valid of", sum(len(r["per_face"]) for r in records))

    if "image" in parts:
        from PIL import Image
        import face_recognition as ref_fr  # reference module (insightface / cv2 stubbed above)
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import _gate_inputs as GI
        r = np.random.Generator(np.random.PCG64(0xFACE0B4D))
        rgb = r.integers(0, 256, (48, 64, 3), dtype=np.uint8)
        gray = r.integers(0, 256, (48, 64), dtype=np.uint8)
        rgba = r.integers(0, 256, (48, 64, 4), dtype=np.uint8)
        Image.fromarray(rgb, "RGB").save(os.path.join(OUT, "image_rgb.png"))
        Image.fromarray(gray, "L").save(os.path.join(OUT, "image_gray.png"))
        Image.fromarray(rgba, "RGBA").save(os.path.join(OUT, "image_rgba.png"))
        want = {"image_rgb.png": sha(rgb), "image_gray.png": sha(np.repeat(gray[:, :, None], 3, axis=2)),
                "image_rgba.png": sha(rgba[..., :3])}
        frame = GI.frame()
        dets = GI.detections()

        class FixedDetector2:
            def detect(self, image):
                assert np.array_equal(image, frame)  # process_image handed process_numpy the RGB frame
                return [{"bbox": d["bbox"].copy(), "landmarks": d["landmarks"].copy(), "det_score": d["det_score"],
                         "pose": None, "age": None, "gender": None} for d in dets]

        png = os.path.join(tmp, "gate_frame.png")
        Image.fromarray(frame, "RGB").save(png)
        fp = ref_fr.FaceProcessor.__new__(ref_fr.FaceProcessor)
        fp.detector, fp.aligner, fp.quality_filter = (FixedDetector2(), ref_fr.FaceAligner(output_size=GI.S),
                                                      ref_fr.FaceQualityFilter())
        runs = {}
        with quiet():
            for ra in (False, True):
                res = fp.process_image(png, return_all=ra)
                runs[str(ra)] = [{"det": next(i for i, d in enumerate(dets)
                                              if np.array_equal(d["landmarks"], r["landmarks"])),
                                  "is_valid": bool(r["is_valid"]), "crop_sha256": sha(r["aligned_face"]),
                                  "blur": float(r["quality_metrics"].get("blur_score", -1.0))} for r in res]
            try:
                fp.process_image(os.path.join(tmp, "missing.png"))
                missing = None
            except ValueError as e:
                missing = str(e).replace(tmp, "<dir>")
        np.savez_compressed(os.path.join(OUT, "image.npz"), decoded_sha256=np.array(json.dumps(want)),
                            process_image=np.array(json.dumps(runs)), missing_error=np.array(missing))
        print("image", {k: len(v) for k, v in runs.items()}, missing)

    if "dropin" in parts:
        import shutil
        from facerecognitionpipeline_amd.gallery_manager import GalleryManager as DropIn
        d = os.path.join(tmp, "dropin")
        os.makedirs(d)
        shutil.copyfile(os.path.join(OUT, "ref_students.pkl"), os.path.join(d, "students.pkl"))
        ours = DropIn(gallery_path=os.path.join(d, "students.pkl"), verbose=False)
        sids = list(ours.students)
        r = np.random.Generator(np.random.PCG64(0xFACE0D1D))

        def unit(n):
            x = r.standard_normal((n, 512)).astype(np.float32)
            return x / np.linalg.norm(x, axis=1, keepdims=True)

        ours.add_student("NEW0001", "Enrolled Through The Drop-In", unit(3), metadata={"source": "frhip"})
        ours.update_embeddings(sids[1], unit(2), mode="append")
        ours.delete_student(sids[2])
        ours.save()
        shutil.copyfile(os.path.join(d, "students.pkl"), os.path.join(OUT, "dropin_students.pkl"))
        with quiet():
            ref = ref_gm.GalleryManager(gallery_path=os.path.join(d, "students.pkl"))  # the reference's load
        ids = list(ref.students)
        recs = [{"student_id": x.student_id, "name": x.name, "num_samples": int(x.num_samples),
                 "enrollment_date": x.enrollment_date, "last_updated": x.last_updated, "metadata": x.metadata,
                 "class": type(x).__module__ + "." + type(x).__name__,
                 "embeddings_sha256": sha(np.asarray(x.embeddings)), "embeddings_dtype": str(x.embeddings.dtype),
                 "template_sha256": sha(np.asarray(x.template_embedding))} for x in ref.students.values()]
        queries = np.concatenate([np.asarray(x.embeddings, np.float32) for x in ref.students.values()])
        gal, idx, sc = search_arrays(ref, queries)
        np.savez_compressed(os.path.join(OUT, "dropin_students.npz"), ids=np.array(ids),
                            records=np.array(json.dumps(recs)), queries_sha256=np.array(sha(queries)),
                            search_idx=idx, search_score=sc, gallery_sha256=np.array(sha(gal.astype(np.float32))))
        print("dropin", len(ids), "students read back by the reference; queries", queries.shape)


if __name__ == "__main__":
    main()
