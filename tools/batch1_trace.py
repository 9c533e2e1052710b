"""Batch-1 IR-101 forwards for a rocprofv3 kernel trace (serving breakdown):
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b1 -o run -- python3 tools/batch1_trace.py
"""
import time, torch, sys, os
sys.path.insert(0, os.getcwd())
from facerecognitionpipeline_amd import weights as W
from facerecognitionpipeline_amd.face_embedder import FaceEmbedder
emb = FaceEmbedder(architecture="ir_101", model_path="synthetic", max_batch=64, graph_batch=0)
crops = torch.from_numpy(W.synthetic_crops(1)).cuda()
for _ in range(30): emb.embed_tensor(crops)
torch.cuda.synchronize()
