"""Python restatement of the XDR server's RDS line formatting (the checker
for fmx_xdr_rds_lines): XDRServer::updateRDS + evaluatePiState
(src/xdr_server.cpp:189-213, 403-457).  Test infrastructure only.  Pinned to
the reference itself: tests/test_host_formats.py checks it (and
fmx_xdr_rds_lines) against the lines the reference's XDRServer, compiled into
oracle/_ref, sends a loopback client (tests/golden/xdr_server.json, and live
when oracle/_ref is built)."""


class PyXdr:
    """XDRServer::updateRDS + evaluatePiState (src/xdr_server.cpp:189-213,
    403-457); ctor state xdr_server.cpp:261-266."""

    def __init__(self):
        self.buf = [0] * 64
        self.err = [0] * 8
        self.fill = 0
        self.pos = 63

    def state(self, value):
        count = correct = 0
        for i in range(self.fill):
            if self.buf[i] == value:
                count += 1
                if (self.err[i // 8] & (1 << (i % 8))) == 0:
                    correct += 1
        if correct >= 2:
            return 0
        if count >= 2 and correct:
            return 1
        if count >= 3:
            return 2
        if count == 2 or correct:
            return 3
        return 4

    def update(self, a, b, c, d, errors):
        out = []
        a_err = (errors >> 6) & 3
        b_err = (errors >> 4) & 3
        self.pos = (self.pos + 1) % 64
        self.buf[self.pos] = a
        if a_err:
            self.err[self.pos // 8] |= 1 << (self.pos % 8)
        else:
            self.err[self.pos // 8] &= ~(1 << (self.pos % 8)) & 0xFF
        if self.fill < 64:
            self.fill += 1
        st = self.state(a)
        if a_err != 3 and st <= 1:
            out.append("P%04X" % a + "?" * min(a_err, 3))
        if b_err == 0:
            out.append("R%04X%04X%04X%02X" % (b, c, d, errors))
        return out
