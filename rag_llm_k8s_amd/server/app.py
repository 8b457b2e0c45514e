"""Flask REST API -- drop-in surface of the reference (/root/reference/llm/rag.py:122-204).

Routes (exact request/response/error contract):
  POST /generate     {"prompt": str} -> 200 {"generated_text", "context"}
                                      | 200 {"generated_text": "No relevant information found in the index."}
                                      | 500 {"error": str}
  POST /query        alias of /generate (BASELINE.json names a "/query" API)
  POST /upload_pdf   multipart "file" -> 200 {"message": "PDF processed and indexed successfully. N chunks created."}
                                       | 400 {"error": "No file part" | "No selected file" | "Invalid file format"}
  GET  /index_info   -> {"total_vectors", "dimension", "total_chunks", "sample_chunks"} | 500 {"error"}
New: GET /healthz (liveness), GET /readyz (weights + index loaded), GET /metrics (Prometheus).
"""
from __future__ import annotations

import logging

from flask import Flask, Response, jsonify, request

from ..utils import metrics

log = logging.getLogger(__name__)


def create_app(service) -> Flask:
    app = Flask("rag_llm_k8s_amd")

    def _generate():
        try:
            data = request.json
            user_prompt = data.get("prompt", "")
            debug = bool(data.get("debug", False))
            out = service.generate(user_prompt, debug=debug)
            metrics.inc("requests", route="generate", status="200")
            return jsonify(out)
        except Exception as e:
            log.error("Error in generate_text: %s", str(e), exc_info=True)
            metrics.inc("requests", route="generate", status="500")
            return jsonify({"error": str(e)}), 500

    app.add_url_rule("/generate", "generate", _generate, methods=["POST"])
    app.add_url_rule("/query", "query", _generate, methods=["POST"])

    @app.route("/upload_pdf", methods=["POST"])
    def upload_pdf():
        if "file" not in request.files:
            return jsonify({"error": "No file part"}), 400
        file = request.files["file"]
        if file.filename == "":
            return jsonify({"error": "No selected file"}), 400
        if file and file.filename.endswith(".pdf"):
            n = service.ingest_pdf_bytes(file.filename, file.read())
            metrics.inc("requests", route="upload_pdf", status="200")
            return jsonify({"message": f"PDF processed and indexed successfully. {n} chunks created."}), 200
        return jsonify({"error": "Invalid file format"}), 400

    @app.route("/index_info", methods=["GET"])
    def index_info():
        try:
            return jsonify(service.index_info())
        except Exception as e:
            log.error("Error in index_info: %s", str(e), exc_info=True)
            return jsonify({"error": str(e)}), 500

    @app.route("/healthz", methods=["GET"])
    def healthz():
        h = service.health()
        return jsonify(h), (200 if h["engine_alive"] else 503)

    @app.route("/readyz", methods=["GET"])
    def readyz():
        h = service.health()
        ok = h["engine_alive"] and h["ready"]
        return jsonify(h), (200 if ok else 503)

    @app.route("/metrics", methods=["GET"])
    def prom_metrics():
        body, ctype = metrics.exposition()
        return Response(body, mimetype=ctype.split(";")[0] if ctype else "text/plain")

    return app
