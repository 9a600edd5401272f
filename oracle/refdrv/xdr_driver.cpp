// xdr_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// The reference's XDR server (src/xdr_server.cpp, compiled UNMODIFIED as part
// of this translation unit: oracle/Makefile puts $(REF)/src on the include
// path and this file includes it) driven from C entry points, so that the
// XDR wire lines fmx_xdr_rds_lines / fmx_xdr_scan_line emit are checked
// against the reference itself:
//   ref_xdr_pi_state   evaluatePiState (xdr_server.cpp:189-213), reachable
//                      here because it sits in this TU's anonymous namespace
//   ref_xdr_session    a started XDRServer on a loopback port, one
//                      authenticated XDR client; the groups go through
//                      XDRServer::updateRDS (:403-457), the scan lines
//                      through pushScanLine (:492-501), and the lines the
//                      server sends the client come back in `out`.
#include "xdr_server.cpp" // the reference source, as it lies under $(REF)/src

#include <openssl/evp.h>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <string>
#include <vector>

namespace refdrv {

std::string sha1_hex(const std::string &s) {
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_MD_CTX *ctx = EVP_MD_CTX_new();
  EVP_DigestInit_ex(ctx, EVP_sha1(), nullptr);
  EVP_DigestUpdate(ctx, s.data(), s.size());
  EVP_DigestFinal_ex(ctx, md, &len);
  EVP_MD_CTX_free(ctx);
  std::string h;
  char b[3];
  for (unsigned i = 0; i < len; ++i) {
    std::snprintf(b, sizeof(b), "%02x", md[i]);
    h += b;
  }
  return h;
}

// one line from the socket (without the newline); false on EOF / timeout
bool read_line(int fd, std::string &buf, std::string &line) {
  for (;;) {
    const size_t p = buf.find('\n');
    if (p != std::string::npos) {
      line = buf.substr(0, p);
      buf.erase(0, p + 1);
      return true;
    }
    char tmp[4096];
    const ssize_t n = recv(fd, tmp, sizeof(tmp), 0);
    if (n <= 0) return false;
    buf.append(tmp, static_cast<size_t>(n));
  }
}

} // namespace refdrv

extern "C" {

int ref_xdr_pi_state(const uint16_t *buf64, const uint8_t *err8, int fill, uint16_t value) {
  std::array<uint16_t, 64> b{};
  std::array<uint8_t, 8> e{};
  for (int i = 0; i < 64; ++i) b[static_cast<size_t>(i)] = buf64[i];
  for (int i = 0; i < 8; ++i) e[static_cast<size_t>(i)] = err8[i];
  return evaluatePiState(b, e, static_cast<uint8_t>(fill), value);
}

// groups: n x {a, b, c, d}, errors[n]; scan: nscan NUL-terminated lines one
// after the other.  Every group goes through updateRDS, then every scan line
// through pushScanLine; out receives the RDS / scan lines the server sent the
// client, '\n'-separated (handshake, state snapshot, the sampling-command
// reply and the periodic signal lines left out).  Returns the bytes written,
// or a negative code (-1 server, -2 connect / auth, -3 timeout, -4 capacity).
int ref_xdr_session(const uint16_t *groups, const uint8_t *errors, int n, const char *scan, int nscan, int port,
                    char *out, int cap) {
  XDRServer srv(static_cast<uint16_t>(port));
  srv.setVerboseLogging(false);
  srv.setPassword("fmx");
  if (!srv.start()) return -1;
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(static_cast<uint16_t>(port));
  sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (connect(fd, reinterpret_cast<sockaddr *>(&sa), sizeof(sa)) != 0) {
    close(fd);
    srv.stop();
    return -2;
  }
  timeval tv{5, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  std::string buf, line;
  int rc = 0;
  std::vector<std::string> got;
  auto fail = [&](int code) {
    close(fd);
    srv.stop();
    return code;
  };
  // XDR handshake (xdr_server.cpp:717-795): salt, SHA1(salt + password),
  // "a2", "o1,0", the state snapshot (its last line is the sampling line)
  if (!refdrv::read_line(fd, buf, line)) return fail(-2);
  const std::string hash = refdrv::sha1_hex(line + "fmx") + "\n";
  send(fd, hash.data(), hash.size(), 0);
  if (!refdrv::read_line(fd, buf, line) || line != "a2") return fail(-2);
  // the longest sampling interval (1 s), so that the periodic signal lines
  // come rarely; its reply ends the snapshot
  const std::string cmd = "I1000,0\n";
  send(fd, cmd.data(), cmd.size(), 0);
  for (;;) {
    if (!refdrv::read_line(fd, buf, line)) return fail(-3);
    if (line == "I1000,0") break;
  }
  // batches of groups (the server queue keeps 256 lines), each closed by two
  // sentinel scan lines.  The client loop (xdr_server.cpp:802-844) sends, per
  // pass, the RDS queue's new lines and then the scan queue's: a pass that
  // read the RDS queue while a batch was still being pushed can send the
  // batch's first sentinel before the batch's tail.  The second sentinel is
  // pushed only after the first has arrived, i.e. after the pass that sent it
  // ended, and every updateRDS of the batch came before that pass's scan read,
  // so the pass that sends the second sentinel reads the whole rest of the
  // batch first: every RDS line of the batch precedes it (no wall-clock wait).
  auto drain_to = [&](const std::string &sentinel) -> bool {
    for (;;) {
      if (!refdrv::read_line(fd, buf, line)) return false;
      if (line == "U" + sentinel) return true;
      if (!line.empty() && line[0] == 'S') {
        // a periodic signal line, right after the periodic "P%04X" line when
        // the server has a debounced PI and RDS within 1.5 s
        // (xdr_server.cpp:848-878; every RDS line here is recent): drop both.
        // An updateRDS P line may carry a '?' suffix; the periodic one never
        if (!got.empty() && got.back().size() == 5 && got.back()[0] == 'P') got.pop_back();
        continue;
      }
      got.push_back(line);
    }
  };
  auto flush = [&](const std::string &s) -> bool {
    srv.pushScanLine(s + "-a");
    if (!drain_to(s + "-a")) return false;
    srv.pushScanLine(s + "-b");
    return drain_to(s + "-b");
  };
  constexpr int kBatch = 100;
  for (int g0 = 0, k = 0; g0 < n; g0 += kBatch, ++k) {
    for (int g = g0; g < std::min(n, g0 + kBatch); ++g)
      srv.updateRDS(groups[4 * g], groups[4 * g + 1], groups[4 * g + 2], groups[4 * g + 3], errors[g]);
    if (!flush("#fmx-batch-" + std::to_string(k))) return fail(-3);
  }
  const char *sp = scan;
  for (int i = 0; i < nscan; ++i) {
    srv.pushScanLine(sp);
    sp += std::strlen(sp) + 1;
    if (i % 4 == 3 || i == nscan - 1) { // the scan queue keeps 8 lines
      const std::string s = "#fmx-scan-" + std::to_string(i);
      srv.pushScanLine(s);
      if (!drain_to(s)) return fail(-3);
    }
  }
  close(fd);
  srv.stop();
  std::string all;
  for (const auto &l : got) all += l + "\n";
  if (static_cast<int>(all.size()) + 1 > cap) return -4;
  std::memcpy(out, all.c_str(), all.size() + 1);
  rc = static_cast<int>(all.size());
  return rc;
}

} // extern "C"
