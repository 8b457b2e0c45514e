"""Drop-in entry point: `python rag.py` (reference CMD, /root/reference/llm/dockerfile_rag:26).

Same startup sequence as /root/reference/llm/rag.py:199-204 -- load the generator from
MODEL_PATH, ensure the index exists, ingest PDF_DIR, serve Flask on 0.0.0.0:5001 -- but the
compute runs on the MI355X-native engine. With TP_SIZE>1 launch one process per GPU
(torchrun --nproc-per-node TP_SIZE llm/rag.py): rank 0 serves HTTP, the other ranks follow
its engine steps (parallel/tp.py).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rag_llm_k8s_amd.server.main import main  # noqa: E402

if __name__ == "__main__":
    main()
