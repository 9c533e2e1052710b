"""Drop-in ``GalleryManager`` whose ``search`` runs on the gfx950 matcher.

Mirrors ``gallery_manager.GalleryManager`` (``gallery_manager.py:53-330``):
student records, template construction (quality filter + mean / median /
weighted_mean + L2) and the ``search(query, top_k) -> [(sid, name, score)]``
contract.  What changes is where the match runs: the reference rebuilds the
G x 512 matrix with ``np.vstack`` on every query (``:177-187``) and sorts all
G scores (``:197``); here the template matrix lives in HBM (uploaded once per
gallery version) and one kernel sequence does renormalise -> fp32 GEMM ->
top-k.  ``search_batch`` exposes the batched form used by the throughput path.

Gallery lifecycle on the device: every mutation is
logged, and the next search brings the HBM copy up to date with row writes /
deletes (``fr_gallery_write_rows`` / ``fr_gallery_delete_rows``) instead of a
full re-upload; ``pending_delta`` gives the same delta to ship to other GPUs
(``distributed.sync_gallery``).  ``add_students_batch`` builds many templates at
once on the GPU (``fr_build_templates``: quality filter + mean / median /
weighted_mean + L2, ``:104-122``, ``:297-317``).

Persistence uses JSON + ``.npz`` (no pickle); ``load_backup`` reads the
reference's ``export_for_backup`` JSON (``:246-270``).
"""
from __future__ import annotations

import copy
import json
import os
import shutil
import threading
import uuid
from dataclasses import dataclass, field
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

SCRIPT_DIR = Path(__file__).resolve().parent


@dataclass
class StudentRecord:
    student_id: str
    name: str
    embeddings: np.ndarray
    template_embedding: np.ndarray
    num_samples: int
    enrollment_date: str
    last_updated: str
    metadata: Dict = field(default_factory=dict)

    def to_dict(self) -> Dict:
        return {"student_id": self.student_id, "name": self.name,
                "embeddings": np.asarray(self.embeddings).tolist(),
                "template_embedding": np.asarray(self.template_embedding).tolist(),
                "num_samples": self.num_samples, "enrollment_date": self.enrollment_date,
                "last_updated": self.last_updated, "metadata": self.metadata or {}}

    @classmethod
    def from_dict(cls, d: Dict) -> "StudentRecord":
        return cls(student_id=d["student_id"], name=d["name"], embeddings=np.array(d["embeddings"]),
                   template_embedding=np.array(d["template_embedding"]), num_samples=d["num_samples"],
                   enrollment_date=d["enrollment_date"], last_updated=d["last_updated"],
                   metadata=d.get("metadata", {}) or {})


def _slice_len(n: int, top_k: int) -> int:
    """How many rows ``argsort(...)[::-1][:top_k]`` keeps (Python slice semantics)."""
    return len(range(n)[:top_k])


MAX_PENDING_OPS = 256  # beyond this a full upload is cheaper than replaying row ops
OP_PUT, OP_DELETE = 0, 1


def _delta_layout(g_old: int, ops) -> List[Tuple[bool, int]]:
    """Final row order after replaying ``ops`` on ``g_old`` rows: per final row, (True, old
    row it keeps) or (False, index into the PUT rows)."""
    src: List[Tuple[bool, int]] = [(True, i) for i in range(g_old)]
    r = 0
    for kind, row in ops:
        if kind == OP_DELETE:
            src.pop(row)
        else:
            if row == len(src):
                src.append((False, r))
            else:
                src[row] = (False, r)
            r += 1
    return src


def apply_gallery_delta(handle: "_lib.Handle", ops: torch.Tensor, rows: torch.Tensor) -> None:
    """Replay a compiled delta on a handle's HBM gallery.  ``ops`` int32 [n,2] of
    (OP_PUT, row) / (OP_DELETE, row); PUTs consume ``rows`` [m,512] in order.

    Without deletes, runs of PUTs to consecutive rows become one write each.  With deletes
    the final layout is computed on the host and the gallery is rebuilt in ONE device pass
    (gather of the surviving rows + the new ones), instead of one tail compaction per
    delete (O(G) each)."""
    ops = ops.cpu().tolist()
    rows = rows.to(handle.device, torch.float32)
    if any(kind == OP_DELETE for kind, _row in ops):
        layout = _delta_layout(handle.gallery_size(), ops)
        E = handle.gallery_read()
        out = torch.empty((len(layout), 512), dtype=torch.float32, device=handle.device)
        keep = [(j, i) for j, (old, i) in enumerate(layout) if old]
        new = [(j, i) for j, (old, i) in enumerate(layout) if not old]
        if keep:
            dst, srcr = (torch.tensor(c, dtype=torch.long, device=handle.device) for c in zip(*keep))
            out[dst] = E[srcr]
        if new:
            dst, srcr = (torch.tensor(c, dtype=torch.long, device=handle.device) for c in zip(*new))
            out[dst] = rows[srcr]
        handle.gallery_replace(out)
        return
    i, r = 0, 0
    while i < len(ops):
        kind, row = ops[i]
        if kind == OP_DELETE:
            handle.gallery_delete_rows(row, 1)
            i += 1
            continue
        j = i + 1
        while j < len(ops) and ops[j][0] == OP_PUT and ops[j][1] == row + (j - i):
            j += 1
        handle.gallery_write_rows(row, rows[r:r + (j - i)])
        r += j - i
        i = j


def apply_gallery_delta_matrix(E: torch.Tensor, ops: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    """Same delta on a plain [G,512] tensor (the semantics of apply_gallery_delta)."""
    E = E.clone()
    r = 0
    for kind, row in ops.cpu().tolist():
        if kind == OP_DELETE:
            E = torch.cat([E[:row], E[row + 1:]])
        elif row == E.shape[0]:
            E = torch.cat([E, rows[r:r + 1].to(E)])
            r += 1
        else:
            E[row] = rows[r].to(E)
            r += 1
    return E


class GalleryManager:
    def __init__(self, gallery_path: Optional[str] = None, aggregation_method: str = "mean", device=None,
                 verbose: bool = True):
        if gallery_path is None:
            gallery_path = str(SCRIPT_DIR / "gallery" / "students.npz")
        self.gallery_path = gallery_path
        self.aggregation_method = aggregation_method
        self.students: Dict[str, StudentRecord] = {}
        self.verbose = verbose
        self._device = torch.device(device) if device is not None else None
        self._handle: Optional[_lib.Handle] = None
        self._version = 0          # bumped by every mutation
        self._device_version = -1  # version the HBM copy holds
        self._ids: List[str] = []  # row order of the HBM copy
        self._uid = uuid.uuid4().hex
        self._pending: Optional[List[Tuple[int, str]]] = None  # row ops since the HBM copy; None = full
        # one lock per manager: mutations, the HBM sync and each search's row -> id resolution
        # are atomic with respect to each other (the reference server shares one GalleryManager
        # across Flask request threads, face_recognition_server.py:1102)
        self._lock = threading.RLock()
        self._save_lock = threading.Lock()  # one save() at a time: snapshot + both files, in order
        os.makedirs(os.path.dirname(gallery_path) or ".", exist_ok=True)
        if os.path.exists(self._arrays_path(gallery_path)):
            self.load()
            self._log(f"Loaded gallery with {len(self.students)} students")
        else:
            self._log("Initialized empty gallery")

    # -- records -------------------------------------------------------------
    def add_student(self, student_id: str, name: str, embeddings: np.ndarray, metadata: Optional[Dict] = None,
                    overwrite: bool = False) -> bool:
        with self._lock:
            if student_id in self.students and not overwrite:
                self._log(f"Student {student_id} already exists. Use overwrite=True to replace.")
                return False
            emb = embeddings.reshape(1, -1) if embeddings.ndim == 1 else embeddings
            now = datetime.now().isoformat()
            self.students[student_id] = StudentRecord(student_id, name, emb, self._aggregate_embeddings(emb),
                                                      len(emb), now, now, metadata or {})
            self._touch((OP_PUT, student_id))
            self._log(f"{'Updated' if overwrite else 'Added'} student: {name} ({student_id}) with {len(emb)} embeddings")
            return True

    def update_embeddings(self, student_id: str, new_embeddings: np.ndarray, mode: str = "append") -> bool:
        with self._lock:
            rec = self.students.get(student_id)
            if rec is None:
                self._log(f"Student {student_id} not found")
                return False
            new = new_embeddings.reshape(1, -1) if new_embeddings.ndim == 1 else new_embeddings
            if mode == "append":
                emb = np.vstack([rec.embeddings, new])
            elif mode == "replace":
                emb = new
            elif mode == "merge":
                emb = self._remove_outliers(np.vstack([rec.embeddings, new]))
            else:
                raise ValueError(f"Unknown mode: {mode}")
            rec.embeddings = emb
            rec.template_embedding = self._aggregate_embeddings(emb)
            rec.num_samples = len(emb)
            rec.last_updated = datetime.now().isoformat()
            self._touch((OP_PUT, student_id))
            return True

    def delete_student(self, student_id: str) -> bool:
        with self._lock:
            if student_id not in self.students:
                self._log(f"Student {student_id} not found")
                return False
            del self.students[student_id]
            self._touch((OP_DELETE, student_id))
            return True

    def add_students_batch(self, entries: Sequence[Tuple[str, str, np.ndarray]], overwrite: bool = False,
                           min_similarity: float = 0.70) -> int:
        """``add_student`` for many students, templates built in one GPU launch
        (``fr_build_templates``).  ``entries``: (student_id, name, embeddings [n_i,512]).
        Returns how many were added (existing ids are skipped unless ``overwrite``)."""
        with self._lock:
            todo = [(sid, name, np.asarray(e, np.float32).reshape(-1, 512)) for sid, name, e in entries
                    if overwrite or sid not in self.students]
            if not todo:
                return 0
            h = self._get_handle()
            offsets = np.zeros(len(todo) + 1, np.int64)
            offsets[1:] = np.cumsum([len(e) for _s, _n, e in todo])
            allemb = torch.from_numpy(np.ascontiguousarray(np.concatenate([e for _s, _n, e in todo]))).to(self.device)
            tpl, _kept = h.build_templates(allemb, offsets, self.aggregation_method, min_similarity)
            tpl = tpl.cpu().numpy()
            now = datetime.now().isoformat()
            for i, (sid, name, e) in enumerate(todo):
                self.students[sid] = StudentRecord(sid, name, e, tpl[i], len(e), now, now, {})
                self._touch((OP_PUT, sid))
            self._log(f"Added {len(todo)} students (templates built on {self.device})")
            return len(todo)

    def get_student(self, student_id: str) -> Optional[StudentRecord]:
        return self.students.get(student_id)

    def get_all_students(self) -> Dict[str, StudentRecord]:
        return self.students

    def get_gallery_embeddings(self) -> Tuple[np.ndarray, List[str]]:
        with self._lock:
            if not self.students:
                return np.array([]), []
            ids = list(self.students.keys())
            return np.vstack([self.students[s].template_embedding for s in ids]), ids

    # -- matching (device) ---------------------------------------------------
    def search(self, query_embedding: np.ndarray, top_k: int = 5) -> List[Tuple[str, str, float]]:
        return self.search_batch(np.asarray(query_embedding).reshape(1, -1), top_k)[0]

    def search_batch(self, queries: np.ndarray, top_k: int = 5) -> List[List[Tuple[str, str, float]]]:
        """search() for every row of ``queries`` [n, 512], one device round trip."""
        q = torch.from_numpy(np.ascontiguousarray(queries, dtype=np.float32)).to(self.device)
        return self.match_resolved(len(queries), top_k, lambda h, k, idx, score: h.match(q, k, idx, score))

    def match_resolved(self, n: int, top_k: int, launch) -> List[List[Tuple[str, str, float]]]:
        """Bring the HBM copy up to date, run ``launch(handle, k, idx, score)`` (any kernel
        sequence that fills idx/score [n,k] with gallery rows), and turn rows into
        ``(sid, name, score)`` -- all under the gallery lock, so a concurrent mutation can
        neither change the rows between the match and their resolution nor make two threads
        replay one delta twice."""
        with self._lock:
            if not self.students:
                return [[] for _ in range(n)]
            k = _slice_len(len(self.students), top_k)
            if k == 0 or n == 0:
                return [[] for _ in range(n)]
            h = self._sync_device()
            idx = torch.empty((n, k), dtype=torch.int32, device=self.device)
            score = torch.empty((n, k), dtype=torch.float32, device=self.device)
            launch(h, k, idx, score)
            idx, score = idx.cpu().numpy(), score.cpu().numpy()
            ids = self._ids
            return [[(ids[i], self.students[ids[i]].name, float(s)) for i, s in zip(ri, rs)]
                    for ri, rs in zip(idx, score)]

    def search_device(self, queries: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Device form: float32 [n,512] on the GPU -> (int32 [n,k] gallery rows, float32 [n,k] scores).
        Row order is ``get_gallery_embeddings()`` order (dict insertion order) at the time of the
        call; a caller that resolves rows while other threads mutate the gallery holds ``_lock``
        across both (or uses :meth:`match_resolved`)."""
        with self._lock:
            h = self._sync_device()
            n = queries.shape[0]
            idx = torch.empty((n, k), dtype=torch.int32, device=self.device)
            score = torch.empty((n, k), dtype=torch.float32, device=self.device)
            h.match(queries.contiguous(), k, idx, score)
            return idx, score

    @property
    def device(self) -> torch.device:
        if self._device is None:
            self._device = torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        return self._device

    def attach_handle(self, handle: "_lib.Handle") -> None:
        """Share an existing handle (e.g. a FaceEmbedder's) so embed+match run in one library state."""
        self._handle = handle
        self._device = handle.device
        self._device_version = -1
        self._pending = None

    def _get_handle(self) -> "_lib.Handle":
        if self._handle is None:
            self._handle = _lib.Handle("ir_50", "adaface", self.device, max_batch=1)
        return self._handle

    def _device_current(self) -> bool:
        """The handle holds exactly this manager's rows at ``_device_version``."""
        return self._handle is not None and self._handle.gallery_tag == (self._uid, self._device_version)

    def pending_delta(self) -> Optional[Tuple[torch.Tensor, torch.Tensor, List[str]]]:
        """Row ops that turn the HBM copy (version ``_device_version``) into the current
        gallery: (ops int32 [n,2], rows f32 [m,512], new row order), or None when only a
        full upload will do (no copy yet, bulk load, too many ops)."""
        if self._pending is None or not self._device_current():
            return None
        ids = list(self._ids)
        pos = {s: i for i, s in enumerate(ids)}
        ops, rows = [], []
        for kind, sid in self._pending:
            if kind == OP_DELETE:
                row = pos.get(sid)
                if row is None:
                    return None
                ops.append((OP_DELETE, row))
                ids.pop(row)
                pos = {s: i for i, s in enumerate(ids)}
            else:
                row = pos.get(sid)
                if row is None:
                    row = len(ids)
                    ids.append(sid)
                    pos[sid] = row
                rec = self.students.get(sid)
                rows.append(np.zeros(512, np.float32) if rec is None
                            else np.asarray(rec.template_embedding, np.float32).reshape(512))
                ops.append((OP_PUT, row))
        if ids != list(self.students.keys()):
            return None
        ops_t = torch.tensor(ops, dtype=torch.int32).reshape(-1, 2)
        rows_t = torch.from_numpy(np.stack(rows)) if rows else torch.zeros((0, 512), dtype=torch.float32)
        return ops_t, rows_t, ids

    def _mark_synced(self, ids: List[str]) -> None:
        self._ids = ids
        self._device_version = self._version
        self._pending = []
        self._handle.gallery_tag = (self._uid, self._version)

    def _sync_device(self) -> "_lib.Handle":
        with self._lock:
            return self._sync_device_locked()

    def _sync_device_locked(self) -> "_lib.Handle":
        h = self._get_handle()
        if self._device_version == self._version and self._device_current():
            return h
        delta = self.pending_delta()
        if delta is None:
            E, ids = self.get_gallery_embeddings()
            h.gallery_set(torch.from_numpy(np.ascontiguousarray(E, dtype=np.float32)).to(self.device))
        else:
            ops, rows, ids = delta
            apply_gallery_delta(h, ops, rows)
        self._mark_synced(ids)
        return h

    # -- persistence ---------------------------------------------------------
    @staticmethod
    def _arrays_path(path: str) -> str:
        root, _ext = os.path.splitext(path)
        return root + ".npz"

    def save(self, path: Optional[str] = None) -> None:
        path = path or self.gallery_path
        # _save_lock orders whole saves (the later snapshot lands last, and no save interleaves its
        # .npz with another's .json); the snapshot itself is taken under the gallery lock, so
        # enrollment is blocked only while it is copied, not while the files are written
        with self._save_lock:
            with self._lock:
                ids = list(self.students.keys())
                arrays = {}
                for i, s in enumerate(ids):
                    arrays[f"e{i}"] = np.array(self.students[s].embeddings)
                    arrays[f"t{i}"] = np.array(self.students[s].template_embedding)
                meta = {"num_students": len(ids), "last_saved": datetime.now().isoformat(), "order": ids,
                        "students": {s: {"student_id": r.student_id, "name": r.name, "num_samples": r.num_samples,
                                         "enrollment_date": r.enrollment_date, "last_updated": r.last_updated,
                                         "metadata": copy.deepcopy(r.metadata)} for s, r in self.students.items()}}
            # both files written to temporaries first and then renamed, so a reader never sees a
            # half-written file (a crash between the two renames can still pair a new .npz with the
            # previous .json; load() then fails on the missing e{i}/t{i} or ids)
            npz, js = self._arrays_path(path), os.path.splitext(path)[0] + ".json"
            with open(npz + ".tmp", "wb") as f:
                np.savez(f, **arrays)
            with open(js + ".tmp", "w") as f:
                json.dump(meta, f, indent=2)
            os.replace(npz + ".tmp", npz)
            os.replace(js + ".tmp", js)

    def load(self, path: Optional[str] = None) -> None:
        with self._lock:
            path = path or self.gallery_path
            arr_path = self._arrays_path(path)
            if not os.path.exists(arr_path):
                self._log(f"Gallery file not found: {arr_path}")
                return
            with open(os.path.splitext(path)[0] + ".json") as f:
                meta = json.load(f)
            arrays = np.load(arr_path)
            self.students = {}
            for i, s in enumerate(meta["order"]):
                m = meta["students"][s]
                self.students[s] = StudentRecord(s, m["name"], arrays[f"e{i}"], arrays[f"t{i}"], m["num_samples"],
                                                 m["enrollment_date"], m["last_updated"], m.get("metadata", {}))
            self._touch()

    def load_backup(self, json_path: str) -> None:
        """Import a reference ``export_for_backup`` JSON (gallery_manager.py:246-270)."""
        with self._lock:
            with open(json_path) as f:
                data = json.load(f)
            self.students = {sid: StudentRecord.from_dict(d) for sid, d in data["students"].items()}
            self._touch()

    def export_for_backup(self, backup_dir: str, backup_name: Optional[str] = None) -> str:
        os.makedirs(backup_dir, exist_ok=True)
        stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
        stem = f"{backup_name}_backup_{stamp}" if backup_name else f"gallery_backup_{stamp}"
        if os.path.exists(self._arrays_path(self.gallery_path)):
            shutil.copy2(self._arrays_path(self.gallery_path), os.path.join(backup_dir, stem + ".npz"))
        out = os.path.join(backup_dir, stem + ".json")
        with self._lock:  # snapshot: to_dict() copies every record into plain lists
            doc = {"backup_date": datetime.now().isoformat(), "backup_name": backup_name,
                   "num_students": len(self.students),
                   "students": {s: r.to_dict() for s, r in self.students.items()}}
        with open(out, "w") as f:
            json.dump(doc, f, indent=2)
        return out

    def get_statistics(self) -> Dict:
        with self._lock:
            recs = list(self.students.values())
        n = len(recs)
        if n == 0:
            return {"num_students": 0, "total_embeddings": 0, "avg_embeddings_per_student": 0}
        total = sum(r.num_samples for r in recs)
        return {"num_students": n, "total_embeddings": total, "avg_embeddings_per_student": total / n,
                "students": [{"id": r.student_id, "name": r.name, "num_samples": r.num_samples,
                              "enrollment_date": r.enrollment_date} for r in recs]}

    # -- template construction (host; offline, KAT-pinned) -------------------
    def _filter_quality_embeddings(self, embeddings: np.ndarray, min_similarity: float = 0.70) -> np.ndarray:
        if len(embeddings) <= 2:
            return embeddings
        sim = embeddings @ embeddings.T
        np.fill_diagonal(sim, 0)
        mean_sim = sim.mean(axis=1)
        kept = embeddings[mean_sim >= min_similarity]
        if len(kept) < 2:
            kept = embeddings[np.argsort(mean_sim)[-2:]]
        return kept

    def _aggregate_embeddings(self, embeddings: np.ndarray) -> np.ndarray:
        if len(embeddings) == 1:
            return embeddings[0]
        e = self._filter_quality_embeddings(embeddings)
        if self.aggregation_method == "median":
            t = np.median(e, axis=0)
        elif self.aggregation_method == "weighted_mean":
            w = (e @ e.T).mean(axis=1)
            t = (e * (w / w.sum())[:, None]).sum(axis=0)
        else:  # 'mean' and any unknown method (reference falls back to mean)
            t = e.mean(axis=0)
        return t / (np.linalg.norm(t) + 1e-8)

    def _remove_outliers(self, embeddings: np.ndarray, threshold: float = 0.7) -> np.ndarray:
        if len(embeddings) <= 2:
            return embeddings
        avg = (embeddings @ embeddings.T).mean(axis=1)
        return embeddings[avg >= np.median(avg) * threshold]

    def _touch(self, op: Optional[Tuple[int, str]] = None) -> None:
        """Bump the version; ``op`` = the row op a device delta replays (None: full upload)."""
        self._version += 1
        if op is None or self._pending is None:
            self._pending = None
        else:
            self._pending.append(op)
            if len(self._pending) > MAX_PENDING_OPS:
                self._pending = None

    def _log(self, msg: str) -> None:
        if self.verbose:
            print(msg)


def build_gallery_matrix(records: Sequence[StudentRecord]) -> np.ndarray:
    """Stack templates in record order (the matrix ``search`` scores against)."""
    return np.vstack([r.template_embedding for r in records]).astype(np.float32)
