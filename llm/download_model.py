"""Model provisioning (initContainer), same CLI/env/layout as /root/reference/llm/download_model.py.

Default behaviour matches the reference: download the 10 named files of
meta-llama/Meta-Llama-3.1-8B-Instruct into /models with HF_TOKEN. Differences:
  * failures exit non-zero (the reference printed and exited 0, so a broken initContainer
    "succeeded", download_model.py:32-33) and the token is never echoed;
  * --embedder also fetches the embedder into /models/<name> (the reference downloaded
    BAAI/bge-m3 from the network at every pod start, rag.py:33);
  * --synthetic writes a random-init checkpoint of the same architecture + a trained
    tokenizer in the same layout, fully offline (tests, benchmarks, air-gapped clusters).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FILES = [
    "config.json",
    "generation_config.json",
    "model-00001-of-00004.safetensors",
    "model-00002-of-00004.safetensors",
    "model-00003-of-00004.safetensors",
    "model-00004-of-00004.safetensors",
    "model.safetensors.index.json",
    "special_tokens_map.json",
    "tokenizer.json",
    "tokenizer_config.json",
]


def download_model(model_name="meta-llama/Meta-Llama-3.1-8B-Instruct", save_directory="/models", embedder=None):
    hf_token = os.environ.get("HF_TOKEN")
    if not hf_token:
        print("Error: Hugging Face token not found in environment variables.")
        return 1
    from huggingface_hub import hf_hub_download, snapshot_download

    try:
        for file in FILES:
            print(f"Downloading file: {file}")
            hf_hub_download(repo_id=model_name, filename=file, local_dir=save_directory, token=hf_token)
        if embedder:
            dst = os.path.join(save_directory, embedder.split("/")[-1])
            print(f"Downloading embedder {embedder} -> {dst}")
            snapshot_download(repo_id=embedder, local_dir=dst, token=hf_token,
                              allow_patterns=["*.json", "*.safetensors", "1_Pooling/*", "*.txt", "*.model"])
        print(f"Model files downloaded successfully to {save_directory}")
        return 0
    except Exception as e:
        print(f"Error downloading model: {str(e)}")
        return 2


def write_synthetic(save_directory, model, embedder, seed=0):
    from rag_llm_k8s_amd.models import encoder as E
    from rag_llm_k8s_amd.models import gpt2 as G2
    from rag_llm_k8s_amd.models import llama as L
    from rag_llm_k8s_amd.utils import synthetic as S

    cfgs = {"llama-3.1-8b": L.llama31_8b, "llama-3.1-70b": L.llama31_70b, "llama-tiny": lambda: L.llama_tiny(vocab=2048)}
    if model == "gpt2":
        G2.write_gpt2_checkpoint(save_directory, G2.GPT2Config(), seed)
    elif model == "gpt2-tiny":
        G2.write_gpt2_checkpoint(save_directory, G2.gpt2_tiny(2048), seed)
    else:
        cfg = cfgs[model]()
        n_shards = 4 if cfg.num_hidden_layers >= 32 else 1
        S.write_llama_checkpoint(save_directory, cfg, seed, n_shards=n_shards)
    if embedder:
        ecfgs = {"all-MiniLM-L6-v2": E.minilm_l6, "bge-large-en-v1.5": E.bge_large_en, "bge-m3": E.bge_m3,
                 "minilm-tiny": lambda: E.EncoderConfig(vocab_size=2048, hidden_size=128, num_hidden_layers=2,
                                                       num_attention_heads=4, intermediate_size=256)}
        S.write_encoder_checkpoint(os.path.join(save_directory, embedder), ecfgs[embedder](), seed)
    print("synthetic checkpoint written to", save_directory)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Meta-Llama-3.1-8B-Instruct")
    ap.add_argument("--out", default=os.environ.get("MODEL_PATH", "/models"))
    ap.add_argument("--embedder", default=os.environ.get("EMBED_REPO"))
    ap.add_argument("--synthetic", action="store_true", help="offline random-init checkpoint")
    ap.add_argument("--arch", default="llama-3.1-8b",
                    help="synthetic architecture: llama-3.1-8b | llama-3.1-70b | llama-tiny | gpt2 | gpt2-tiny")
    ap.add_argument("--synthetic-embedder", default="all-MiniLM-L6-v2")
    a = ap.parse_args()
    if a.synthetic:
        return write_synthetic(a.out, a.arch, a.synthetic_embedder)
    return download_model(a.model, a.out, a.embedder)


if __name__ == "__main__":
    sys.exit(main())
