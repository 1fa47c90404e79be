// HTTP/1.1 parsing helpers shared by the server/blocking client (http.cpp) and the event-driven
// client (http_async.cpp).
#pragma once

#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace die {
namespace http_detail {

bool iequals(std::string_view a, std::string_view b);
std::string_view trim(std::string_view s);
void set_nonblock(int fd);
// TCP_NODELAY, and the fixed socket buffers when the peer is on loopback (core/http.cpp).
void set_nodelay(int fd, bool loopback_peer = false);
// SO_RCVBUF the kernel granted the first loopback socket (-1: none yet / buffers off).
int sock_buf_effective();
// Header block (start line excluded) -> lower-cased (name, value) pairs.
void parse_headers(std::string_view block, std::vector<std::pair<std::string, std::string>>& out);
// Complete chunked body at `data`: bytes consumed, 0 if incomplete, -1 malformed, -2 over max_out.
long dechunk(std::string_view data, std::string& out, size_t max_out);

}  // namespace http_detail
}  // namespace die
