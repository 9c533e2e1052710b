"""Device gallery lifecycle against the oracle and the reference's KATs.

* ``fr_build_templates`` vs ``GalleryManager._aggregate_embeddings`` restated
  (oracle/reference_path.py, gallery_manager.py:104-122, 297-317) and the reference's
  own templates of its committed backups (tests/golden/backup_*.npz).
* incremental HBM sync (row writes / deletes) vs a full upload after random
  enrollment changes.
"""
import os

import numpy as np
import pytest
import torch

from oracle import reference_path as rp

pytestmark = pytest.mark.gpu
BACKUPS = ("adaface_ir_101", "adaface_ir_50", "arcface_ir_101", "arcface_ir_50")


@pytest.fixture(scope="module")
def handle():
    from facerecognitionpipeline_amd import _lib
    return _lib.Handle("ir_50", "adaface", torch.device("cuda", 0), max_batch=1)


@pytest.mark.parametrize("name", BACKUPS)
def test_build_templates_backup_kat(handle, name, golden_dir):
    f = np.load(os.path.join(golden_dir, f"backup_{name}.npz"))
    E = f["embeddings"]                                   # [students, 8, 512] from the reference's JSON
    S, n = E.shape[:2]
    tpl, kept = handle.build_templates(torch.from_numpy(E.reshape(-1, 512)).cuda(), np.arange(S + 1) * n, "mean")
    tpl = tpl.cpu().numpy()
    want_kept = [len(rp.filter_quality_embeddings(e)) for e in E]
    assert kept.cpu().numpy().tolist() == want_kept
    assert np.abs(tpl - f["ref_template"]).max() <= 1e-7        # reference GalleryManager output
    assert np.abs(tpl - f["stored_template"]).max() <= 1e-7     # the committed templates


def test_search_on_reference_gallery_pickle(tmp_path, golden_dir):
    """The reference's own gallery file (tests/golden/ref_students.pkl, written by the reference
    GalleryManager.save, gallery_manager.py:207-210) loaded through the restricted unpickler and
    searched on the GPU: every stored sample's top-5 equals the reference search of the same
    templates (backup_adaface_ir_101.npz, gallery_manager.py:189-205), scores within 1e-6."""
    import shutil
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    f = np.load(os.path.join(golden_dir, "backup_adaface_ir_101.npz"))
    shutil.copyfile(os.path.join(golden_dir, "ref_students.pkl"), tmp_path / "students.pkl")
    gm = GalleryManager(gallery_path=str(tmp_path / "students.pkl"), device="cuda:0", verbose=False)
    q = f["embeddings"].reshape(-1, 512)
    res = gm.search_batch(q, top_k=5)
    ids = [str(s) for s in f["student_ids"]]
    got_idx = np.array([[ids.index(sid) for sid, _n, _s in r] for r in res])
    got_sc = np.array([[sc for _sid, _n, sc in r] for r in res], dtype=np.float32)
    assert np.array_equal(got_idx, f["search_idx"])
    assert np.abs(got_sc - f["search_score"]).max() <= 1e-6
    assert res[0][0][1] == gm.students[res[0][0][0]].name
    # single-query form, as FaceMatcher.match_single_face calls it
    one = gm.search(q[9], top_k=3)
    assert [ids.index(s) for s, _n, _sc in one] == f["search_idx"][9][:3].tolist()


def test_search_on_dropin_written_gallery_equals_reference(tmp_path, golden_dir):
    """A gallery saved by this module (tests/golden/dropin_students.pkl) and read by the REFERENCE
    GalleryManager gives the reference's search results (tools/make_golden.py dropin); the GPU
    search of the same file gives the same top-5 rows, scores within 1e-6."""
    import shutil
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    fx = np.load(os.path.join(golden_dir, "dropin_students.npz"))
    shutil.copyfile(os.path.join(golden_dir, "dropin_students.pkl"), tmp_path / "students.pkl")
    gm = GalleryManager(gallery_path=str(tmp_path / "students.pkl"), device="cuda:0", verbose=False)
    ids = [str(s) for s in fx["ids"]]
    q = np.concatenate([np.asarray(r.embeddings, np.float32) for r in gm.students.values()])
    res = gm.search_batch(q, top_k=5)
    assert np.array_equal(np.array([[ids.index(s) for s, _n, _sc in r] for r in res]), fx["search_idx"])
    assert np.abs(np.array([[sc for _s, _n, sc in r] for r in res]) - fx["search_score"]).max() <= 1e-6


@pytest.mark.parametrize("method", ["mean", "median", "weighted_mean"])
def test_build_templates_random_vs_oracle(handle, method):
    """Ragged students (1..40 samples), clusters loose enough that the 0.70 filter drops
    rows and sometimes falls back to the top-2 rows."""
    rng = np.random.default_rng(3)
    sizes = rng.integers(1, 41, size=64)
    sizes[:4] = [1, 2, 3, 40]
    embs = []
    for i, n in enumerate(sizes):
        base = rng.normal(size=512)
        spread = 0.4 + 1.2 * (i % 4) / 3
        e = base[None] + spread * rng.normal(size=(n, 512))
        e /= np.linalg.norm(e, axis=1, keepdims=True)
        embs.append(e.astype(np.float32))
    off = np.concatenate([[0], np.cumsum(sizes)])
    tpl, kept = handle.build_templates(torch.from_numpy(np.concatenate(embs)).cuda(), off, method)
    tpl, kept = tpl.cpu().numpy(), kept.cpu().numpy()
    fallbacks = 0
    for i, e in enumerate(embs):
        filt = rp.filter_quality_embeddings(e) if len(e) > 1 else e
        assert kept[i] == len(filt)
        fallbacks += len(e) > 2 and len(filt) == 2
        want = rp.aggregate_template(e, method)
        tol = 1e-7 if method == "mean" else 1e-6
        assert np.abs(tpl[i] - want).max() <= tol, (i, len(e), method)
    assert fallbacks > 0 and (kept < sizes).any()


def test_build_templates_rejects_bad_offsets(handle):
    e = torch.zeros((4, 512), device="cuda")
    with pytest.raises(ValueError):
        handle.build_templates(e, [0, 2, 2, 4])        # empty student
    with pytest.raises(ValueError):
        handle.build_templates(e, [1, 4])              # offsets[0] != 0
    with pytest.raises(ValueError):
        handle.build_templates(torch.zeros((1025, 512), device="cuda"), [0, 1025])


def test_incremental_sync_equals_full_upload(tmp_path):
    from facerecognitionpipeline_amd import _lib
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    h = _lib.Handle("ir_50", "adaface", torch.device("cuda", 0), max_batch=1)
    calls = {"full": 0}
    orig = h.gallery_set

    def counting_set(E, tag=None):
        calls["full"] += 1
        return orig(E, tag)

    h.gallery_set = counting_set
    gm = GalleryManager(gallery_path=str(tmp_path / "a" / "s.npz"), device="cuda:0", verbose=False)
    gm.attach_handle(h)
    rng = np.random.default_rng(9)

    def emb(n):
        e = rng.normal(size=(n, 512)).astype(np.float32)
        return e / np.linalg.norm(e, axis=1, keepdims=True)

    for i in range(50):
        gm.add_student(f"S{i}", f"N{i}", emb(3))
    q = emb(16)
    gm.search_batch(q, 5)
    assert calls["full"] == 1
    nxt = 50
    for _round in range(20):
        for _ in range(int(rng.integers(1, 8))):
            ids = list(gm.students)
            op = rng.integers(0, 4)
            if op == 0:
                gm.add_student(f"S{nxt}", "x", emb(int(rng.integers(1, 6))))
                nxt += 1
            elif op == 1:
                gm.add_student(ids[rng.integers(len(ids))], "y", emb(4), overwrite=True)
            elif op == 2:
                gm.update_embeddings(ids[rng.integers(len(ids))], emb(2))
            else:
                gm.delete_student(ids[rng.integers(len(ids))])
        got = gm.search_batch(q, 5)
        dev = h.gallery_read().cpu().numpy()
        assert np.array_equal(dev, np.asarray(gm.get_gallery_embeddings()[0], np.float32))
        fresh = GalleryManager(gallery_path=str(tmp_path / "b" / "s.npz"), device="cuda:0", verbose=False)
        fresh.students = dict(gm.students)
        fresh._touch()
        assert fresh.search_batch(q, 5) == got
    assert calls["full"] == 1          # every change after the first upload went as row ops


def test_add_students_batch_matches_add_student(tmp_path):
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    rng = np.random.default_rng(4)
    entries = []
    for i in range(40):
        base = rng.normal(size=512)
        e = base[None] + 0.5 * rng.normal(size=(int(rng.integers(1, 12)), 512))
        entries.append((f"S{i}", f"N{i}", (e / np.linalg.norm(e, axis=1, keepdims=True)).astype(np.float32)))
    a = GalleryManager(gallery_path=str(tmp_path / "a" / "s.npz"), device="cuda:0", verbose=False)
    b = GalleryManager(gallery_path=str(tmp_path / "b" / "s.npz"), device="cuda:0", verbose=False)
    assert a.add_students_batch(entries) == 40
    assert a.add_students_batch(entries[:3]) == 0              # existing ids skipped
    for sid, name, e in entries:
        b.add_student(sid, name, e)
    Ea, Eb = a.get_gallery_embeddings()[0], b.get_gallery_embeddings()[0]
    assert np.abs(Ea - Eb).max() <= 1e-7
    q = np.stack([e[0] for _s, _n, e in entries])
    assert [[r[0] for r in x] for x in a.search_batch(q, 3)] == [[r[0] for r in x] for x in b.search_batch(q, 3)]


def test_concurrent_mutation_and_search_stay_consistent(tmp_path):
    """searches racing enrollment changes on one GalleryManager (the reference's Flask
    threads share one, face_recognition_server.py:1102).  Every result must be the host search of
    SOME consistent gallery state: each returned (sid, score) pair equals q . template(sid) of
    that student at some version, and the HBM copy ends equal to the host matrix."""
    import threading
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    gm = GalleryManager(gallery_path=str(tmp_path / "c" / "s.npz"), device="cuda:0", verbose=False)
    rng = np.random.default_rng(17)

    def unit(n):
        e = rng.normal(size=(n, 512)).astype(np.float32)
        return e / np.linalg.norm(e, axis=1, keepdims=True)

    base = unit(40)
    for i in range(40):
        gm.add_student(f"S{i}", f"N{i}", base[i])
    history = {f"S{i}": [base[i]] for i in range(40)}  # every template each sid ever had
    q = base[:8] + 0.05 * unit(8)
    errors = []
    stop = threading.Event()

    def searcher():
        try:
            while not stop.is_set():
                for r, row in zip(q, gm.search_batch(q, 3)):
                    for sid, name, sc in row:
                        best = min(abs(float(np.dot(r / np.linalg.norm(r), t)) - sc) for t in history[sid])
                        if best > 1e-5:
                            errors.append((sid, sc, best))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=searcher) for _ in range(4)]
    for t in threads:
        t.start()
    nxt = 40
    for step in range(150):
        ids = list(gm.students)
        op = step % 3
        if op == 0 and len(ids) > 10:
            gm.delete_student(ids[int(rng.integers(len(ids)))])
        elif op == 1:
            e = unit(1)[0]
            history.setdefault(f"S{nxt}", []).append(e)
            gm.add_student(f"S{nxt}", "x", e)
            nxt += 1
        else:
            sid = ids[int(rng.integers(len(ids)))]
            e = unit(1)[0]
            history[sid].append(e)
            gm.add_student(sid, "y", e, overwrite=True)
    stop.set()
    for t in threads:
        t.join(30)
    assert not errors, errors[:5]
    gm.search_batch(q, 3)
    dev = gm._get_handle().gallery_read().cpu().numpy()
    assert np.array_equal(dev, np.asarray(gm.get_gallery_embeddings()[0], np.float32))


def test_batched_delete_compaction(tmp_path):
    """A sync with many deletes rebuilds the rows in one device pass (apply_gallery_delta) and
    ends equal to the host matrix."""
    from facerecognitionpipeline_amd.gallery_manager import GalleryManager
    gm = GalleryManager(gallery_path=str(tmp_path / "d" / "s.npz"), device="cuda:0", verbose=False)
    rng = np.random.default_rng(3)
    E = rng.normal(size=(300, 512)).astype(np.float32)
    for i in range(300):
        gm.add_student(f"S{i}", "n", E[i])
    gm.search_batch(E[:2], 1)
    for i in range(0, 300, 3):
        gm.delete_student(f"S{i}")
    gm.add_student("S1", "m", E[0], overwrite=True)
    gm.add_student("NEW", "m", E[5])
    assert gm.pending_delta() is not None
    res = gm.search_batch(E[:4], 1)
    dev = gm._get_handle().gallery_read().cpu().numpy()
    assert np.array_equal(dev, np.asarray(gm.get_gallery_embeddings()[0], np.float32))
    assert res[0][0][0] == "S1" and res[2][0][0] == "S2"


def test_match_scores_over_2gib_are_chunked(handle):
    """fr_match_topk keeps each score matrix below 2 GiB (the conv epilogue's 32-bit offsets): a
    600k-row gallery and 1,000 queries (2.4 GB of scores) run in query chunks.  Queries are
    gallery rows, so each one's top-1 is its own row at score 1 with a wide margin."""
    g = torch.Generator(device="cuda").manual_seed(7)
    G, n = 600_000, 1_000
    E = torch.randn(G, 512, device="cuda", generator=g)
    E = E / E.norm(dim=1, keepdim=True)
    handle.gallery_set(E)
    rows = torch.randint(0, G, (n,), device="cuda", generator=g)
    idx = torch.empty((n, 2), dtype=torch.int32, device="cuda")
    score = torch.empty((n, 2), dtype=torch.float32, device="cuda")
    handle.match(E[rows].contiguous(), 2, idx, score)
    torch.cuda.synchronize()
    assert torch.equal(idx[:, 0].long(), rows)
    assert (score[:, 0] - 1).abs().max().item() < 1e-5 and score[:, 1].max().item() < 0.5
    handle.gallery_set(torch.empty((0, 512), device="cuda"))


@pytest.mark.parametrize("G", [1, 7, 64, 1000, 4099])
def test_small_batch_match_vs_reference(handle, G):
    """Serving-sized match (n <= 16: normalisation fused into the scores launch, then top-k) and
    the batched path (n = 17: l2norm + score GEMM + top-k) vs ``search``'s arithmetic in float64
    (gallery_manager.py:195-197).  Ties are planted (duplicate rows): they must rank by
    descending row, the documented policy.  Run twice: reused workspaces."""
    g = np.random.default_rng(G)
    E = g.standard_normal((G, 512)).astype(np.float32)
    E /= np.linalg.norm(E, axis=1, keepdims=True)
    if G >= 7:
        E[G // 2] = E[1]  # a tie with row 1
    handle.gallery_set(torch.from_numpy(E).cuda())
    Q = g.standard_normal((17, 512)).astype(np.float32)
    Q[2] = E[min(1, G - 1)] * 3.0        # exact-tie query (G >= 7): rows 1 and G // 2 score the same
    for n in (1, 5, 16, 17):
        k = min(8 if n <= 16 else 5, G)
        q = torch.from_numpy(Q[:n]).cuda()
        for _ in range(2):
            idx = torch.empty((n, k), dtype=torch.int32, device="cuda")
            sc = torch.empty((n, k), dtype=torch.float32, device="cuda")
            handle.match(q, k, idx, sc)
            torch.cuda.synchronize()
            qn = Q[:n].astype(np.float64) / (np.linalg.norm(Q[:n].astype(np.float64), axis=1, keepdims=True) + 1e-8)
            S = qn @ E.astype(np.float64).T
            assert np.abs(sc.cpu().numpy() - np.take_along_axis(S, idx.cpu().numpy().astype(np.int64), 1)).max() < 2e-6
            order = np.argsort(-S, axis=1, kind="stable")[:, :k]
            got = idx.cpu().numpy()
            for r in range(n):
                srt = np.sort(S[r])[::-1]
                top = srt[:k + 1]
                margin = np.min(np.abs(np.diff(top))) if top.size > 1 else 1.0
                if margin > 1e-5:
                    assert np.array_equal(got[r], order[r]), (n, r)
            if n >= 3 and G >= 7:
                assert set(got[2][:2].tolist()) == {1, G // 2} and got[2][0] == max(1, G // 2)
    handle.gallery_set(torch.empty((0, 512), device="cuda"))
