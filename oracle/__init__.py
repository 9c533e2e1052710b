"""CPU oracle for the embed + match hot path — TEST INFRASTRUCTURE ONLY.

Nothing in ``facerecognitionpipeline_amd`` may import this package.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg use it, and only as the checker / CPU baseline, never as the product.

Contents
--------
adaface_net      restatement of upstream AdaFace ``net.py`` (absent from the
                 reference; imported at ``face_embedder.py:3,11,49``) as a
                 plain PyTorch-CPU fp32 module with the same state-dict keys.
reference_path   restatement of the reference's own numpy/torch glue:
                 ``FaceEmbedder.preprocess`` / ``extract_embedding[s_batch]``
                 (``face_embedder.py:93-182``) and ``GalleryManager.search`` /
                 ``_aggregate_embeddings`` (``gallery_manager.py:104-122,
                 177-205, 297-317``).

Pinning
-------
* ``reference_path`` search/aggregation is pinned against the reference's
  committed gallery backups (``gallery/backups/*.json``) through
  ``tests/golden/backup_*.npz`` (template KAT <=4.5e-8, 184/184 self top-1).
* ``adaface_net`` + ``reference_path`` embed is pinned against golden vectors
  produced by importing the reference ``FaceEmbedder`` / ``GalleryManager`` in
  the build container (``tools/make_golden.py``).  The network itself comes
  from upstream AdaFace (mk-minchul/AdaFace ``net.py``, unpinned, not
  vendored), so its arithmetic is pinned to the reference's *wrapper* only;
  against upstream weights it is "parity unpinned" (no checkpoints exist
  offline).  See DESIGN.md §Oracle.
"""
