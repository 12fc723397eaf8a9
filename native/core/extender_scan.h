// Zero-copy scan of kube-scheduler ExtenderArgs.
//
// With nodeCacheCapable=false (the reference's extender setting,
// scheduler-configmap.yaml:61-79) every filter / prioritize call carries the
// FULL Node object of every candidate node: ~7 KB each, ~9 MB per call at
// 1,250 nodes (10,000 GPUs).  Building a DOM for that and re-serialising the
// surviving nodes costs ~250 ms per call — three times the p99 budget.  The
// extender only needs each node's metadata.name, and the filter reply must
// echo the passing Node objects unchanged, so this scanner
//   * parses the (small) "pod" value into a DOM,
//   * walks "nodes"/"Nodes" -> "items" recording each item's byte span and
//     its metadata.name (string-aware brace skipping at memory speed),
//   * leaves the reply to splice the original item bytes back together.
// Anything unexpected (malformed text, escapes in a node name) makes scan()
// return false and the caller falls back to the full parser.
#pragma once
#include <string>
#include <string_view>
#include <vector>

#include "json.h"

namespace kgwe {

struct NodeSpan {
  std::string name;
  size_t begin = 0, end = 0;  // [begin, end) of the item's JSON text
};

struct ExtenderArgsScan {
  Json pod;                            // "pod" / "Pod"
  bool have_nodes = false;             // "nodes" / "Nodes" object present (full Node objects)
  std::vector<NodeSpan> nodes;         // its items
  std::vector<std::string> nodenames;  // "nodenames" / "NodeNames"
};

bool scan_extender_args(std::string_view text, ExtenderArgsScan* out);

// The names of the items of {"nodes": {"items": [...]}} in an
// ExtenderFilterResult / ExtenderArgs text (for callers that only need names).
bool scan_node_names(std::string_view text, std::vector<std::string>* names);

}  // namespace kgwe
