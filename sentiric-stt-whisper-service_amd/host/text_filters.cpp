#include "text_filters.h"

#include <algorithm>
#include <cctype>
#include <cstring>

namespace mwx_host {

namespace {

const char* const kWs = " \t\n\r\f\v";

// Phrase list of the reference filter (data, src/utils.h:223-259).
const char* const kBanned[] = {
    "altyazı", "Altyazı", "ALTYAZI", "sesli betimleme", "Sesli betimleme", "senkron", "Senkron",
    "www.", ".com", "izlediğiniz için", "İzlediğiniz için", "İZLEDİĞİNİZ İÇİN", "teşekkürler",
    "Teşekkürler", "TEŞEKKÜRLER", "teşekkür ederim", "Teşekkür ederim", "TEŞEKKÜR EDERİM",
    "thank you", "Thank you", "Thanks for watching", "abone ol", "Abone ol", "videoyu beğen",
    "bir sonraki videoda", "devam edecek", "Devam edecek", "transcription:", "subtitle:", "2分",
    "ご視聴", "I'm going to go", "Okay.", "Bye.", "Ahem.", "Ahem", "Umarım", "umarım"};

// Short noises compared after punctuation stripping (src/utils.h:295-301).
const char* const kNoises[] = {"Hıhı", "hıhı", "Pffft", "pffft", "Ehem", "ehem", "Hmm", "hmm",
                               "Aa",   "aa",   "Ah",    "ah",    "Oh",   "oh",   "Eh",   "eh"};

// ::tolower on each byte (bytes >= 0x80 of UTF-8 text are left as they are in
// the "C" locale, which is what the reference's std::transform does).
std::string ascii_lower(std::string s) {
  for (char& ch : s) ch = (char)std::tolower((unsigned char)ch);
  return s;
}

std::string strip_punct(std::string s) {
  while (!s.empty() && std::ispunct((unsigned char)s.back())) s.pop_back();
  size_t i = 0;
  while (i < s.size() && std::ispunct((unsigned char)s[i])) ++i;
  return s.substr(i);
}

}  // namespace

std::string trim_ws(const std::string& s) {
  const size_t a = s.find_first_not_of(kWs);
  if (a == std::string::npos) return "";
  const size_t b = s.find_last_not_of(kWs);
  return s.substr(a, b - a + 1);
}

bool is_hallucination(const std::string& raw_text) {
  const std::string text = trim_ws(raw_text);
  if (text.size() < 2) return true;  // empty or a single byte
  if (text.find_first_not_of(" \t\n\v\f\r.,?!") == std::string::npos) return true;
  if ((text.front() == '[' && text.back() == ']') || (text.front() == '(' && text.back() == ')'))
    return true;
  const std::string lower = ascii_lower(text);
  // phrases longer than 4 bytes: substring match on the text or its lowercase
  for (const char* ph : kBanned) {
    if (std::strlen(ph) > 4 &&
        (lower.find(ph) != std::string::npos || text.find(ph) != std::string::npos))
      return true;
  }
  const std::string stripped = strip_punct(lower);
  const std::string stripped_orig = strip_punct(text);
  // phrases up to 6 bytes: whole-text match after punctuation stripping
  for (const char* ph : kBanned) {
    if (std::strlen(ph) <= 6 && (stripped == ascii_lower(ph) || stripped_orig == ph)) return true;
  }
  for (const char* nz : kNoises)
    if (stripped == nz || stripped_orig == nz) return true;
  return false;
}

}  // namespace mwx_host
