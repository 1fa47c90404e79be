// Prometheus text exposition (format 0.0.4) of a JSON stats document: GET /metrics on the worker
// and the gateway serves the same numbers as /health and /stats, flattened for a scraper.
// Every numeric or boolean leaf becomes one untyped sample named <prefix>_<path> (path segments
// joined by '_', anything outside [a-zA-Z0-9_] mapped to '_', array elements as an `index`
// label); strings become labels of a constant `<prefix>_info 1` sample.  An addition beyond the
// reference, which only has the JSON routes.
#pragma once

#include <string>

#include "json.h"

namespace die {

// `labels`: preformatted label pairs added to every sample, e.g. `node="worker1"` (may be empty).
std::string prometheus_text(const Json& stats, const std::string& prefix, const std::string& labels);

}  // namespace die
