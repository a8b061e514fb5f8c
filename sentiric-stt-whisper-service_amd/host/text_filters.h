// Service-level text filters applied to every decoded segment.
//
// Restates the behaviour of the reference's hallucination filter
// (src/utils.h:214-306, sentiric::utils::is_hallucination) and trim
// (src/utils.h:205-210): a segment is dropped when, after trimming ASCII
// whitespace, it is empty or one byte long, consists only of whitespace and
// ".,?!", is fully bracketed by [] or (), contains (case-sensitively, or in an
// ASCII-lowercased copy) one of the longer banned phrases, equals one of the
// short banned phrases / noise words once leading and trailing ASCII
// punctuation is stripped.
#pragma once

#include <string>

namespace mwx_host {

std::string trim_ws(const std::string& s);
bool is_hallucination(const std::string& raw_text);

}  // namespace mwx_host
