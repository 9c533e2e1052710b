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

Persistence: ``save`` writes the reference's own gallery file -- ``<stem>.pkl``
= ``pickle.dump(dict[str, gallery_manager.StudentRecord])`` with the same
fields (``:207-210``), so the reference's ``load`` and every reference tool
reads enrollments made here -- plus one ``.npz`` (every array and, as a JSON
string, every record's fields and the signature of the ``.pkl`` written with
it: a single atomic file) and the reference's informational ``.json`` sidecar
(same keys as ``:211-229``).  ``load`` reads the ``.npz`` or, when the ``.pkl``
no longer matches the signature the ``.npz`` recorded (the reference app wrote
it since), the ``.pkl``, through a restricted unpickler that resolves only
numpy's array reconstruction and the reference's ``StudentRecord`` (mapped onto
this module's dataclass) and executes nothing else from the file; an unreadable
or foreign pickle raises, it never turns into an empty gallery.
``export_for_backup`` copies the gallery files (``:246-270``: ``FileNotFoundError``
when there is none) and ``load_backup`` reads its JSON.
"""
from __future__ import annotations

import copy
import errno
import hashlib
import importlib
import json
import logging
import os
import pickle
import shutil
import tempfile
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


# -- the reference's gallery pickle (gallery_manager.py:207-210 dump, :234-244 load) ----------
class _PickledRecord:
    """Receives the attributes of a pickled reference ``StudentRecord``; no code of the file runs
    (pickle's NEWOBJ + BUILD only create the instance and fill its ``__dict__``)."""


# globals a reference gallery pickle may name: numpy's array / dtype / scalar reconstruction
# (numpy 1.x ``numpy.core`` and 2.x ``numpy._core`` spellings) and the reference's record class
# (``gallery_manager.StudentRecord``, or ``__main__.StudentRecord`` when the reference module ran
# as a script, gallery_manager.py:333-362)
_NUMPY_GLOBALS = {
    ("numpy", "ndarray"), ("numpy", "dtype"),
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy.core.numeric", "_frombuffer"), ("numpy._core.numeric", "_frombuffer"),
}
_RECORD_GLOBALS = {("gallery_manager", "StudentRecord"), ("__main__", "StudentRecord")}


class _GalleryUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _RECORD_GLOBALS:
            return _PickledRecord
        if (module, name) in _NUMPY_GLOBALS:
            if module == "numpy":
                return getattr(np, name)
            tail = module.split(".", 2)[2]  # multiarray / numeric, under whichever core this numpy has
            for core in ("numpy._core", "numpy.core"):
                try:
                    return getattr(importlib.import_module(f"{core}.{tail}"), name)
                except (ImportError, AttributeError):
                    continue
        raise pickle.UnpicklingError(f"gallery pickle names a global outside the whitelist: {module}.{name}")


def _float_array(v, what: str) -> np.ndarray:
    if not isinstance(v, np.ndarray) or v.dtype.kind != "f":
        raise ValueError(f"gallery pickle: {what} is not a float array")
    return v


def load_reference_pickle(path: str) -> Dict[str, "StudentRecord"]:
    """The ``Dict[str, StudentRecord]`` the reference's ``save`` pickled, as this module's records.
    Raises ``pickle.UnpicklingError`` for a global outside the whitelist and ``ValueError`` for
    anything that is not such a dict of records."""
    with open(path, "rb") as f:
        obj = _GalleryUnpickler(f).load()
    if not isinstance(obj, dict):
        raise ValueError(f"gallery pickle {path}: top level is {type(obj).__name__}, not a dict of StudentRecord")
    out: Dict[str, StudentRecord] = {}
    for sid, r in obj.items():
        if not isinstance(r, _PickledRecord):
            raise ValueError(f"gallery pickle {path}: entry {sid!r} is {type(r).__name__}, not a StudentRecord")
        d = r.__dict__
        try:
            emb = _float_array(d["embeddings"], f"{sid} embeddings")
            tpl = _float_array(d["template_embedding"], f"{sid} template_embedding")
            rec = StudentRecord(str(d["student_id"]), str(d["name"]), emb, tpl, int(d["num_samples"]),
                                str(d["enrollment_date"]), str(d["last_updated"]), d.get("metadata") or {})
        except KeyError as e:
            raise ValueError(f"gallery pickle {path}: record {sid!r} lacks field {e}") from None
        if not isinstance(rec.metadata, dict):
            raise ValueError(f"gallery pickle {path}: record {sid!r} metadata is not a dict")
        out[sid] = rec
    return out


# -- writing the reference's gallery pickle ------------------------------------------------------
class _RefStudentRecord:
    """Stand-in that pickles as the reference's ``gallery_manager.StudentRecord`` (never instantiated)."""


_RECORD_FIELDS = ("student_id", "name", "embeddings", "template_embedding", "num_samples", "enrollment_date",
                  "last_updated", "metadata")


class _ReferencePickler(pickle._Pickler):
    """``pickle.dump(self.students)`` as the reference's ``save`` runs it (gallery_manager.py:207-210):
    each record is a ``gallery_manager.StudentRecord`` rebuilt by NEWOBJ + BUILD from its eight
    dataclass fields in declaration order; numpy arrays pickle through numpy's own reduction.  The
    reference's module need not be importable here: the class is written by name."""

    def __init__(self, f):
        super().__init__(f, protocol=pickle.DEFAULT_PROTOCOL)

    def _save_record(self, obj):
        # what save_reduce writes for copyreg.__newobj__(cls) + state, with the reference's class
        self.save(_RefStudentRecord)
        self.save(())
        self.write(pickle.NEWOBJ)
        self.memoize(obj)
        self.save({k: getattr(obj, k) for k in _RECORD_FIELDS})
        self.write(pickle.BUILD)

    dispatch = dict(pickle._Pickler.dispatch)

    def save_global(self, obj, name=None):
        if obj is not _RefStudentRecord:
            return super().save_global(obj, name)
        if self.proto >= 4:
            self.save("gallery_manager")
            self.save("StudentRecord")
            self.write(pickle.STACK_GLOBAL)
        else:
            self.write(pickle.GLOBAL + b"gallery_manager\nStudentRecord\n")
        self.memoize(obj)


_ReferencePickler.dispatch[StudentRecord] = _ReferencePickler._save_record


def dump_reference_pickle(students: Dict[str, "StudentRecord"], f) -> None:
    """Write ``students`` in the reference's gallery-file format (readable by its ``load``)."""
    _ReferencePickler(f).dump(students)


def _file_signature(path: str) -> Optional[Dict]:
    """{"size", "sha256"} of a file, or None when it does not exist."""
    try:
        h = hashlib.sha256()
        n = 0
        with open(path, "rb") as f:
            for chunk in iter(lambda: f.read(1 << 20), b""):
                h.update(chunk)
                n += len(chunk)
        return {"size": n, "sha256": h.hexdigest()}
    except FileNotFoundError:
        return None


_log = logging.getLogger(__name__)
# the process umask, read once at import (os.umask can only be read by setting it)
_UMASK = os.umask(0o022)
os.umask(_UMASK)


def _atomic_write(path: str, write) -> None:
    """``write(fileobj)`` into a uniquely named temporary in ``path``'s directory, then rename it
    over ``path``: readers see the old file or the new one, and concurrent savers (other managers,
    other processes) never share a temporary.  The file keeps the mode of the one it replaces, or
    gets 0666 & ~umask when new -- as a plain ``open(path, "w")`` would (mkstemp creates 0600)."""
    fd, tmp = tempfile.mkstemp(prefix=os.path.basename(path) + ".", suffix=".tmp", dir=os.path.dirname(path) or ".")
    try:
        with os.fdopen(fd, "wb") as f:
            write(f)
        try:
            mode = os.stat(path).st_mode & 0o7777
        except FileNotFoundError:
            mode = 0o666 & ~_UMASK
        os.chmod(tmp, mode)
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


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
            gallery_path = str(SCRIPT_DIR / "gallery" / "students.pkl")  # the reference's default name (:57-58)
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
        if self._source(gallery_path) is not None:
            self.load()  # raises on a file it cannot read: never an empty gallery in its place
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

    @staticmethod
    def _pickle_path(path: str) -> str:
        root, _ext = os.path.splitext(path)
        return root + ".pkl"

    @staticmethod
    def _recorded_pickle(npz: str):
        """The ``.pkl`` signature a ``save`` recorded in its ``.npz`` ({"size", "sha256"}, or None
        when it wrote no ``.pkl`` and none existed), or "unknown" for ``.npz`` files of earlier
        rounds, which recorded nothing."""
        try:
            with np.load(npz) as arrays:
                if "meta" not in arrays.files:
                    return "unknown"
                meta = json.loads(str(arrays["meta"]))
        except (OSError, ValueError):
            return "unknown"
        return meta.get("pkl", "unknown")

    @classmethod
    def _source(cls, path: str) -> Optional[Tuple[str, str]]:
        """What ``load(path)`` reads: ("npz", file) -- this module's save -- or ("pkl", file) -- the
        reference's ``pickle.dump(self.students)`` (gallery_manager.py:207-210), or None.  When both
        exist, the ``.npz`` unless the ``.pkl`` differs from the one the ``.npz`` was saved with
        (its size + SHA-256, recorded by ``save``): then the reference app has written the
        ``.pkl`` since, and it is the newer gallery.  File times are not consulted (a copy or a
        checkout resets them), except for ``.npz`` files of earlier rounds that recorded no
        signature.  The choice is logged at warning level whenever both files exist."""
        npz, pkl = cls._arrays_path(path), cls._pickle_path(path)
        have_npz, have_pkl = os.path.exists(npz), os.path.exists(pkl)
        if have_npz and have_pkl:
            rec = cls._recorded_pickle(npz)
            if rec == "unknown":
                pick = "pkl" if os.path.getmtime(pkl) > os.path.getmtime(npz) else "npz"
                why = "the .npz records no .pkl signature (an earlier save); the newer file wins"
            elif rec is not None and _file_signature(pkl) == rec:
                pick, why = "npz", "the .pkl is the one saved with it"
            else:
                pick, why = "pkl", "the .pkl changed after the .npz was saved (written by another program)"
            _log.warning("gallery %s: both %s and %s exist; loading the .%s: %s", path, os.path.basename(npz),
                         os.path.basename(pkl), pick, why)
            return (pick, pkl if pick == "pkl" else npz)
        if have_npz:
            return "npz", npz
        if have_pkl:
            return "pkl", pkl
        return None

    def save(self, path: Optional[str] = None, reference_pickle: bool = True) -> None:
        """Write the gallery: ``<stem>.pkl`` in the reference's own format (gallery_manager.py:207-210;
        ``reference_pickle=False`` leaves any ``.pkl`` at the path as it is), ``<stem>.npz``
        (templates, samples, every record field and the ``.pkl``'s signature: the whole gallery in
        one file) and the reference's informational ``<stem>.json`` sidecar (:211-229).  Each file
        is replaced atomically; the ``.pkl`` goes first, so a save cut short leaves an ``.npz``
        whose recorded signature no longer matches, and ``load`` takes the newer ``.pkl``."""
        path = path or self.gallery_path
        # _save_lock orders whole saves of this manager (the later snapshot lands last); unique
        # temporaries keep saves of other managers / processes from mixing; the snapshot itself is
        # taken under the gallery lock, so enrollment is blocked only while it is copied
        with self._save_lock:
            with self._lock:
                ids = list(self.students.keys())
                arrays = {}
                for i, s in enumerate(ids):
                    arrays[f"e{i}"] = np.array(self.students[s].embeddings)
                    arrays[f"t{i}"] = np.array(self.students[s].template_embedding)
                now = datetime.now().isoformat()
                fields = {s: {"student_id": r.student_id, "name": r.name, "num_samples": r.num_samples,
                              "enrollment_date": r.enrollment_date, "last_updated": r.last_updated,
                              "metadata": copy.deepcopy(r.metadata)} for s, r in self.students.items()}
                snap = None
                if reference_pickle:  # records sharing nothing mutable with the live ones
                    snap = {s: StudentRecord(r.student_id, r.name, arrays[f"e{i}"], arrays[f"t{i}"], r.num_samples,
                                             r.enrollment_date, r.last_updated, fields[s]["metadata"])
                            for i, (s, r) in enumerate(self.students.items())}
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            pkl = self._pickle_path(path)
            if snap is not None:
                _atomic_write(pkl, lambda f: dump_reference_pickle(snap, f))
            meta = {"format": "frhip-gallery-1", "order": ids, "students": fields, "pkl": _file_signature(pkl)}
            arrays["meta"] = np.array(json.dumps(meta))
            _atomic_write(self._arrays_path(path), lambda f: np.savez(f, **arrays))
            sidecar = {"num_students": len(ids), "last_saved": now, "students": fields}
            _atomic_write(os.path.splitext(path)[0] + ".json",
                          lambda f: f.write(json.dumps(sidecar, indent=2).encode()))

    def load(self, path: Optional[str] = None) -> None:
        """Load ``<stem>.npz`` or the reference's ``<stem>.pkl`` (``_source``); a path with neither
        logs and keeps the current records, as the reference does (gallery_manager.py:237-239)."""
        with self._lock:
            path = path or self.gallery_path
            src = self._source(path)
            if src is None:
                self._log(f"Gallery file not found: {path}")
                return
            kind, fpath = src
            if kind == "pkl":
                self.students = load_reference_pickle(fpath)
            else:
                with np.load(fpath) as arrays:
                    if "meta" in arrays.files:
                        meta = json.loads(str(arrays["meta"]))
                    else:  # a round-4 save: fields in the .json beside it
                        with open(os.path.splitext(fpath)[0] + ".json") as f:
                            meta = json.load(f)
                    students = {}
                    for i, s in enumerate(meta["order"]):
                        m = meta["students"][s]
                        students[s] = StudentRecord(s, m["name"], arrays[f"e{i}"], arrays[f"t{i}"],
                                                    m["num_samples"], m["enrollment_date"], m["last_updated"],
                                                    m.get("metadata", {}) or {})
                self.students = students
            self._touch()

    def load_backup(self, json_path: str) -> None:
        """Import a reference ``export_for_backup`` JSON (gallery_manager.py:246-270)."""
        with self._lock:
            with open(json_path) as f:
                data = json.load(f)
            self.students = {sid: StudentRecord.from_dict(d) for sid, d in data["students"].items()}
            self._touch()

    def export_for_backup(self, backup_dir: str, backup_name: Optional[str] = None) -> str:
        """gallery_manager.py:246-270: copy the gallery file(s) -- the reference-format ``.pkl`` and
        this module's ``.npz``, whichever exist -- into ``backup_dir`` as ``<name>_backup_<time>.*``,
        then write the JSON export of every record.  With no gallery file at ``gallery_path`` it
        raises ``FileNotFoundError`` before writing anything, as the reference's ``shutil.copy2``
        does.  Returns the JSON's path."""
        os.makedirs(backup_dir, exist_ok=True)
        stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
        stem = f"{backup_name}_backup_{stamp}" if backup_name else f"gallery_backup_{stamp}"
        files = [f for f in (self._pickle_path(self.gallery_path), self._arrays_path(self.gallery_path))
                 if os.path.exists(f)]
        if not files:
            raise FileNotFoundError(errno.ENOENT, os.strerror(errno.ENOENT), self.gallery_path)
        for f in files:
            shutil.copy2(f, os.path.join(backup_dir, stem + os.path.splitext(f)[1]))
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
