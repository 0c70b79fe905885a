// ConnectedComponentsExample (example/ConnectedComponentsExample.java:49-169) on the
// C++ host mirror: default stream (k, k+2) for k = 1..100 with event time 100*k ms,
// or a whitespace-separated edge file; prints every Merger emission.
// Usage: connected_components_example [<edges path> <merge window ms>]
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

#include "gelly_streaming.hpp"

using namespace gelly;

int main(int argc, char** argv) {
  int64_t mergeWindowTime = 1000;  // :78
  EdgeStream<int64_t, NullValue> s;
  if (argc == 3) {
    std::ifstream in(argv[1]);
    std::string line;
    while (std::getline(in, line)) {  // :109-118, split on whitespace
      std::istringstream ls(line);
      int64_t a, b;
      if (ls >> a >> b) s.edges.push_back({a, b, NullValue{}});
    }
    mergeWindowTime = std::stoll(argv[2]);
  } else if (argc != 1) {
    std::fprintf(stderr, "Usage: connected_components_example <input edges path> <merge window time (ms)>\n");
    return 1;
  } else {
    for (int64_t k = 1; k <= 100; ++k) {  // :121-139
      s.edges.push_back({k, k + 2, NullValue{}});
      s.timestamps.push_back(k * 100);
    }
  }
  SimpleEdgeStream<int64_t, NullValue> edges(s);
  ConnectedComponents<NullValue> cc(mergeWindowTime);
  edges.aggregate(cc, [](const DisjointSetRef& ds) { std::printf("%s\n", ds->toString().c_str()); });
  return 0;
}
