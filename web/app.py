"""Streamlit chat UI (reference web/app.py contract: POST {LLM_SERVICE_URL}/generate {"prompt"} ->
{"generated_text"}). Unchanged request/response contract; adds a request timeout and an optional
view of the retrieved context."""
import os

import requests
import streamlit as st

LLM_SERVICE_URL = os.getenv("LLM_SERVICE_URL", "http://llm-service:80")
TIMEOUT_S = float(os.getenv("LLM_TIMEOUT_S", "300"))

st.title("RAG-Enhanced LLM Chat Interface")
prompt = st.text_input("Enter your prompt:", "")
show_ctx = st.checkbox("Show retrieved context", value=False)

if st.button("Generate"):
    if not prompt:
        st.warning("Please enter a prompt.")
    else:
        try:
            r = requests.post(f"{LLM_SERVICE_URL}/generate", json={"prompt": prompt}, timeout=TIMEOUT_S)
        except requests.RequestException as e:
            st.error(f"Request failed: {e}")
        else:
            if r.status_code == 200:
                body = r.json()
                st.write("Generated response:")
                st.write(body["generated_text"])
                if show_ctx and body.get("context"):
                    with st.expander("Context"):
                        st.text(body["context"])
            else:
                st.error(f"Error: {r.status_code}, {r.text}")

st.write("This interface uses the Meta-Llama-3.1-8B-Instruct model served on AMD Instinct MI355X.")
