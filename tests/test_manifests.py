"""T6: k8s manifests keep the reference's drop-in surface and add the MI355X bits."""
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    with open(os.path.join(ROOT, path)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def test_llm_deployment_surface():
    (d,) = load("llm/ragdeploy.yaml")
    assert d["kind"] == "Deployment" and d["metadata"]["name"] == "llm-deployment"
    spec = d["spec"]["template"]["spec"]
    assert d["spec"]["selector"]["matchLabels"] == {"app": "llm-app"}
    (init,) = spec["initContainers"]
    assert init["name"] == "download-model"
    env = {e["name"]: e for e in init["env"]}
    assert env["HF_TOKEN"]["valueFrom"]["secretKeyRef"] == {"name": "hf-token", "key": "HF_TOKEN"}
    assert "echo" not in " ".join(init.get("args", []) + init.get("command", [])).split("$HF_TOKEN")[0][-30:]
    (c,) = spec["containers"]
    assert c["image"] == "localhost:5003/all-server:v1"
    assert [p["containerPort"] for p in c["ports"]] == [5001]
    mounts = {m["mountPath"]: m["name"] for m in c["volumeMounts"]}
    assert mounts["/models"] == "model-storage" and mounts["/pdfs"] == "pdf-storage"
    vols = {v["name"]: v for v in spec["volumes"]}
    assert vols["model-storage"]["persistentVolumeClaim"]["claimName"] == "llm-model-pvc"
    assert vols["pdf-storage"]["persistentVolumeClaim"]["claimName"] == "pdf-pvc"
    assert vols["download-script"]["configMap"]["name"] == "download-script-configmap"
    assert c["resources"]["limits"]["amd.com/gpu"] == 1
    assert c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz"


def test_services_pvcs_secret_upload_web():
    (s,) = load("llm/service.yaml")
    assert s["metadata"]["name"] == "llm-service" and s["spec"]["type"] == "LoadBalancer"
    assert s["spec"]["selector"] == {"app": "llm-app"}
    assert (s["spec"]["ports"][0]["port"], s["spec"]["ports"][0]["targetPort"]) == (80, 5001)
    pv = {p["metadata"]["name"]: p for p in load("llm/pvc.yaml")}
    assert pv["llm-model-pvc"]["spec"]["accessModes"] == ["ReadWriteOnce"]
    assert pv["llm-model-pvc"]["spec"]["resources"]["requests"]["storage"] == "100Gi"
    assert pv["pdf-pvc"]["spec"]["accessModes"] == ["ReadWriteMany"]
    assert pv["pdf-pvc"]["spec"]["resources"]["requests"]["storage"] == "50Gi"
    (sec,) = load("llm/secret.yaml")
    assert sec["metadata"]["name"] == "hf-token" and "HF_TOKEN" in sec["stringData"]
    (up,) = load("llm/upload.yaml")
    assert up["metadata"]["name"] == "pdf-upload-pod"
    assert up["spec"]["volumes"][0]["persistentVolumeClaim"]["claimName"] == "pdf-pvc"
    (wd,) = load("web/deploy.yaml")
    assert wd["metadata"]["name"] == "streamlit-rag-app"
    wc = wd["spec"]["template"]["spec"]["containers"][0]
    assert wc["ports"][0]["containerPort"] == 8501
    assert any(e["name"] == "LLM_SERVICE_URL" for e in wc["env"])
    (ws,) = load("web/service.yaml")
    assert ws["metadata"]["name"] == "streamlit-app"
    assert (ws["spec"]["ports"][0]["port"], ws["spec"]["ports"][0]["targetPort"]) == (80, 8501)


def test_tp8_variant():
    pvc, d, svc = load("deploy/k8s/ragdeploy-tp8.yaml")
    c = d["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    assert "--nproc-per-node" in c["command"]
    assert {e["name"]: e["value"] for e in c["env"]}["TP_SIZE"] == "8"
    # can run beside llm/ragdeploy.yaml: distinct selector, Service and model PVC; same init container
    (base,) = load("llm/ragdeploy.yaml")
    (base_svc,) = load("llm/service.yaml")
    sel = d["spec"]["selector"]["matchLabels"]
    assert sel != base["spec"]["selector"]["matchLabels"]
    assert not set(base_svc["spec"]["selector"].items()) <= set(d["spec"]["template"]["metadata"]["labels"].items())
    assert set(svc["spec"]["selector"].items()) <= set(d["spec"]["template"]["metadata"]["labels"].items())
    assert svc["metadata"]["name"] == "llm-service-tp8" and svc["spec"]["ports"][0]["targetPort"] == 5001
    vols = {v["name"]: v for v in d["spec"]["template"]["spec"]["volumes"]}
    assert vols["model-storage"]["persistentVolumeClaim"]["claimName"] == pvc["metadata"]["name"] != "llm-model-pvc"
    assert vols["download-script"]["configMap"]["name"] == "download-script-configmap"
    assert d["spec"]["template"]["spec"]["initContainers"][0]["name"] == "download-model"


def test_dockerfile_has_no_baked_token():
    with open(os.path.join(ROOT, "llm/dockerfile_rag")) as f:
        txt = f.read()
    assert "ENV HF_TOKEN" not in txt and "gfx950" in txt
