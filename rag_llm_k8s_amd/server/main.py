"""Server process main (single GPU or one rank of a TP group)."""
from __future__ import annotations

import logging
import os

import torch

from ..config import RagConfig
from ..utils.metrics import setup_logging

log = logging.getLogger("rag")


def main(argv=None):
    cfg = RagConfig.from_env()
    setup_logging(cfg.log_level)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        from ..parallel.tp import run_tp_server

        return run_tp_server(cfg, rank, world)
    if cfg.resolved_device().startswith("cuda"):
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    from .app import create_app
    from .builder import build_service

    svc = build_service(cfg)
    svc.store.ensure_exists()
    processed = svc.ingest_directory()
    if processed == 0:
        log.warning("No PDF files were processed. The index might be empty.")
    svc.ready = True
    app = create_app(svc)
    app.run(host=cfg.host, port=cfg.port, threaded=True)


if __name__ == "__main__":
    main()
