"""Chunking, prompt construction and answer post-processing (byte-exact reference contract).

References:
  split_text                      /root/reference/llm/rag.py:39-45
  process_pdf page concatenation  /root/reference/llm/rag.py:47-52
  SYSTEM_MESSAGE                  /root/reference/llm/rag.py:35-37
  context / prompt template       /root/reference/llm/rag.py:163-169
  answer post-processing          /root/reference/llm/rag.py:173-174
"""
from __future__ import annotations

SYSTEM_MESSAGE = """You are a helpful assistant. Answer the user's question based ONLY on the given context.
If the context doesn't contain relevant information to the specific question, say 'I don't have enough information to answer that specific question.'
Do not make up information or use general knowledge outside of the given context."""

NO_RESULTS = "No relevant information found in the index."


def split_text(text: str, chunk_size: int = 1000, overlap: int = 200):
    """Word windows of `chunk_size` starting every `chunk_size - overlap` words. A trailing
    window is always emitted, even when fully contained in the previous one."""
    words = text.split()
    step = chunk_size - overlap
    if step <= 0:
        raise ValueError("chunk_size must exceed overlap")
    return [" ".join(words[i:i + chunk_size]) for i in range(0, len(words), step)]


def build_context(results, context_k: int = 3) -> str:
    """results: list of (metadata dict, squared-L2 distance) ascending."""
    ctx = ""
    for doc, score in results[:context_k]:
        ctx += f"Document '{doc['filename']}' (chunk {doc['chunk_id']}, score: {score:.4f}): {doc['text']}\n\n"
    return ctx


def build_prompt(context: str, user_prompt: str) -> str:
    return f"{SYSTEM_MESSAGE}\n\nContext: {context}\n\nUser: {user_prompt}\n\nChatbot:"


def postprocess(decoded_full_sequence: str) -> str:
    return decoded_full_sequence.split("Chatbot:")[-1].strip()


def chunk_metadata(filename: str, chunks):
    return [{"filename": filename, "chunk_id": i, "text": c} for i, c in enumerate(chunks)]
