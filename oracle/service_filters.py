"""CPU restatement of the reference service's result post-processing —
TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker of
sentiric-stt-whisper-service_amd/host/).

Follows:
  * sentiric::utils::trim / is_hallucination  (reference src/utils.h:205-306)
  * SttEngine::transcribe result loop          (reference src/stt_engine.cpp:258-337):
    hallucination filter, tokens with id >= eot skipped, average token p over
    the kept tokens < 0.40 drops the segment (only when tokens were kept).
Operates on bytes (the reference works on std::string bytes; ASCII-only
tolower / ispunct as in the "C" locale). Parity unpinned: the reference ships
no tests or fixtures for these functions.
"""
from __future__ import annotations

import string
from typing import List

WS = b" \t\n\r\x0c\x0b"
PUNCT = set(string.punctuation.encode())
BANNED = [s.encode() for s in [
    "altyazı", "Altyazı", "ALTYAZI", "sesli betimleme", "Sesli betimleme", "senkron", "Senkron",
    "www.", ".com", "izlediğiniz için", "İzlediğiniz için", "İZLEDİĞİNİZ İÇİN", "teşekkürler",
    "Teşekkürler", "TEŞEKKÜRLER", "teşekkür ederim", "Teşekkür ederim", "TEŞEKKÜR EDERİM",
    "thank you", "Thank you", "Thanks for watching", "abone ol", "Abone ol", "videoyu beğen",
    "bir sonraki videoda", "devam edecek", "Devam edecek", "transcription:", "subtitle:", "2分",
    "ご視聴", "I'm going to go", "Okay.", "Bye.", "Ahem.", "Ahem", "Umarım", "umarım"]]
NOISES = [s.encode() for s in ["Hıhı", "hıhı", "Pffft", "pffft", "Ehem", "ehem", "Hmm", "hmm",
                               "Aa", "aa", "Ah", "ah", "Oh", "oh", "Eh", "eh"]]


def trim(b: bytes) -> bytes:
    return b.strip(WS)


def lower(b: bytes) -> bytes:
    return bytes(c + 32 if 65 <= c <= 90 else c for c in b)


def strip_punct(b: bytes) -> bytes:
    i, j = 0, len(b)
    while j > i and b[j - 1] in PUNCT:
        j -= 1
    while i < j and b[i] in PUNCT:
        i += 1
    return b[i:j]


def is_hallucination(raw: bytes) -> bool:
    t = trim(raw)
    if len(t) < 2:
        return True
    if all(c in b" \t\n\x0b\x0c\r.,?!" for c in t):
        return True
    if (t[:1] == b"[" and t[-1:] == b"]") or (t[:1] == b"(" and t[-1:] == b")"):
        return True
    lo = lower(t)
    for ph in BANNED:
        if len(ph) > 4 and (ph in lo or ph in t):
            return True
    st, so = strip_punct(lo), strip_punct(t)
    for ph in BANNED:
        if len(ph) <= 6 and (st == lower(ph) or so == ph):
            return True
    return any(st == nz or so == nz for nz in NOISES)


def postprocess(segments, eot: int, token_text) -> List[dict]:
    """segments: list of (text_bytes, t0, t1, [(id, p, t0, t1), ...])."""
    out = []
    for text, t0, t1, toks in segments:
        if is_hallucination(text):
            continue
        kept = [(token_text(i), p, a, b) for i, p, a, b in toks if i < eot]
        avg = float(sum(p for _, p, _, _ in kept) / len(kept)) if kept else 0.0
        if kept and avg < 0.40:
            continue
        out.append({"text": text, "t0": t0, "t1": t1, "prob": avg, "tokens": kept})
    return out
