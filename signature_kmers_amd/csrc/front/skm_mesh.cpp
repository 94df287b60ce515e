// skm_mesh.cpp -- see skm_mesh.h.
#include "skm_mesh.h"

#include <signal.h>
#include <sys/prctl.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

namespace skmf {

namespace {

bool send_all(int fd, const void* p, uint64_t n) {
    const char* c = static_cast<const char*>(p);
    while (n) {
        const ssize_t k = ::send(fd, c, std::min<uint64_t>(n, 1u << 20), MSG_NOSIGNAL);
        if (k <= 0) return false;
        c += k;
        n -= (uint64_t)k;
    }
    return true;
}

bool recv_all(int fd, void* p, uint64_t n) {
    char* c = static_cast<char*>(p);
    while (n) {
        const ssize_t k = ::recv(fd, c, std::min<uint64_t>(n, 1u << 20), 0);
        if (k <= 0) return false;
        c += k;
        n -= (uint64_t)k;
    }
    return true;
}

// one framed message (u64 length + bytes) to every peer, each on its own thread, while the
// caller receives; the per-peer senders never wait on each other, so no cycle can block
template <class SendFn, class RecvFn>
int exchange(const Mesh& m, SendFn payload, RecvFn sink) {
    std::vector<std::thread> th;
    std::vector<int> ok(m.world, 1);
    for (int q = 0; q < m.world; ++q) {
        if (q == m.rank) continue;
        th.emplace_back([&, q]() {
            const auto [p, n] = payload(q);
            const uint64_t len = n;
            ok[q] = send_all(m.fd[q], &len, 8) && send_all(m.fd[q], p, n);
        });
    }
    int rc = 0;
    for (int q = 0; q < m.world; ++q) {
        if (q == m.rank) continue;
        uint64_t len = 0;
        if (!recv_all(m.fd[q], &len, 8)) {
            rc = -1;
            continue;
        }
        void* dst = sink(q, len);
        if (!dst) {
            rc = -1;
            std::vector<char> junk(len);
            recv_all(m.fd[q], junk.data(), len);
            continue;
        }
        if (!recv_all(m.fd[q], dst, len)) rc = -1;
    }
    for (auto& t : th) t.join();
    for (int q = 0; q < m.world; ++q)
        if (!ok[q]) rc = -1;
    return rc;
}

int t_alltoallv(void* ctx, const void* send, const uint64_t* scnt, const uint64_t* soff, void* recv,
                const uint64_t* rcnt, const uint64_t* roff) {
    const Mesh& m = *static_cast<Mesh*>(ctx);
    const char* s = static_cast<const char*>(send);
    char* r = static_cast<char*>(recv);
    if (scnt[m.rank]) std::memcpy(r + roff[m.rank], s + soff[m.rank], scnt[m.rank]);
    return exchange(
        m, [&](int q) { return std::pair<const void*, uint64_t>(s + soff[q], scnt[q]); },
        [&](int q, uint64_t len) -> void* { return len == rcnt[q] ? r + roff[q] : nullptr; });
}

int t_allreduce(void* ctx, void* data, uint64_t count, int op) {
    const Mesh& m = *static_cast<Mesh*>(ctx);
    const uint64_t es = op == 0 ? 4 : 1;
    std::vector<std::vector<uint8_t>> all(m.world);
    const int rc = exchange(
        m, [&](int) { return std::pair<const void*, uint64_t>(data, count * es); },
        [&](int q, uint64_t len) -> void* {
            if (len != count * es) return nullptr;
            all[q].resize(len);
            return all[q].data();
        });
    if (rc) return rc;
    for (int q = 0; q < m.world; ++q) {  // u32 sums wrap mod 2^32 and max commute: any order
        if (q == m.rank) continue;
        if (op == 0) {
            auto* a = static_cast<uint32_t*>(data);
            const auto* b = reinterpret_cast<const uint32_t*>(all[q].data());
            for (uint64_t i = 0; i < count; ++i) a[i] += b[i];
        } else {
            auto* a = static_cast<uint8_t*>(data);
            for (uint64_t i = 0; i < count; ++i) a[i] = std::max(a[i], all[q][i]);
        }
    }
    return 0;
}

int t_allgatherv(void* ctx, const void* send, void* recv, const uint64_t* bytes) {
    const Mesh& m = *static_cast<Mesh*>(ctx);
    std::vector<uint64_t> off(m.world + 1, 0);
    for (int q = 0; q < m.world; ++q) off[q + 1] = off[q] + bytes[q];
    char* r = static_cast<char*>(recv);
    if (bytes[m.rank]) std::memcpy(r + off[m.rank], send, bytes[m.rank]);
    return exchange(
        m, [&](int) { return std::pair<const void*, uint64_t>(send, bytes[m.rank]); },
        [&](int q, uint64_t len) -> void* { return len == bytes[q] ? r + off[q] : nullptr; });
}

}  // namespace

skm_transport Mesh::transport() {
    skm_transport t{};
    t.ctx = this;
    t.alltoallv = t_alltoallv;
    t.allreduce = t_allreduce;
    t.allgatherv = t_allgatherv;
    return t;
}

bool mesh_fork(int world, Mesh& m, std::string& err) {
    m.world = world;
    m.rank = 0;
    m.fd.assign(world, -1);
    if (world == 1) return true;
    std::vector<std::vector<int>> sv(world, std::vector<int>(2 * world, -1));  // [p][2q..]: pair (p, q), p < q
    for (int p = 0; p < world; ++p)
        for (int q = p + 1; q < world; ++q) {
            int s[2];
            if (socketpair(AF_UNIX, SOCK_STREAM, 0, s) != 0) {
                err = "socketpair failed";
                return false;
            }
            sv[p][2 * q] = s[0];
            sv[p][2 * q + 1] = s[1];
        }
    std::vector<int> pw(world, -1), pr(world, -1);
    for (int q = 1; q < world; ++q) {
        int pp[2];
        if (pipe(pp) != 0) {
            err = "pipe failed";
            return false;
        }
        pr[q] = pp[0];
        pw[q] = pp[1];
    }
    std::fflush(nullptr);
    int me = 0;
    for (int q = 1; q < world; ++q) {
        const pid_t pid = fork();
        if (pid < 0) {
            err = "fork failed";
            return false;
        }
        if (pid == 0) {
            me = q;
            // a child blocked in a collective must not outlive rank 0 (which exits on any failure)
            prctl(PR_SET_PDEATHSIG, SIGTERM);
            if (getppid() == 1) _exit(1);
            break;
        }
        m.children.push_back(pid);
    }
    m.rank = me;
    // keep this rank's ends, close the rest
    for (int p = 0; p < world; ++p)
        for (int q = p + 1; q < world; ++q) {
            if (p == me) {
                m.fd[q] = sv[p][2 * q];
                close(sv[p][2 * q + 1]);
            } else if (q == me) {
                m.fd[p] = sv[p][2 * q + 1];
                close(sv[p][2 * q]);
            } else {
                close(sv[p][2 * q]);
                close(sv[p][2 * q + 1]);
            }
        }
    for (int q = 1; q < world; ++q) {
        if (me == 0) {
            close(pr[q]);
            m.id_pipes.resize(world, -1);
            m.id_pipes[q] = pw[q];
        } else {
            close(pw[q]);
            if (q == me)
                m.id_pipe = pr[q];
            else
                close(pr[q]);
        }
    }
    if (me != 0) m.children.clear();
    return true;
}

bool Mesh::share_id(uint8_t id[128], std::string& err) {
    if (world == 1) return true;
    if (rank == 0) {
        for (int q = 1; q < world; ++q)
            if (write(id_pipes[q], id, 128) != 128) {
                err = "cannot send the communicator id to rank " + std::to_string(q);
                return false;
            }
        return true;
    }
    uint64_t got = 0;
    while (got < 128) {
        const ssize_t k = read(id_pipe, id + got, 128 - got);
        if (k <= 0) {
            err = "rank 0 exited before sharing the communicator id";
            return false;
        }
        got += (uint64_t)k;
    }
    return true;
}

void Mesh::watch_children() {
    if (rank != 0 || children.empty() || watching) return;
    watching = std::make_shared<std::atomic<bool>>(true);
    std::thread([kids = children, on = watching]() {
        while (on->load()) {
            for (size_t i = 0; i < kids.size(); ++i) {
                siginfo_t si{};
                // WNOWAIT: the child stays waitable for wait_children
                if (waitid(P_PID, (id_t)kids[i], &si, WEXITED | WNOHANG | WNOWAIT) != 0 || si.si_pid == 0) continue;
                if (si.si_code == CLD_EXITED && si.si_status == 0) continue;
                if (!on->load()) return;
                std::fprintf(stderr, "rank %zu failed; stopping the other ranks\n", i + 1);
                for (pid_t k : kids) kill(k, SIGTERM);
                std::fflush(nullptr);
                _exit(1);
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(100));
        }
    }).detach();
}

bool Mesh::wait_children(std::string& err) {
    if (watching) watching->store(false);
    bool ok = true;
    for (size_t i = 0; i < children.size(); ++i) {
        int st = 0;
        if (waitpid(children[i], &st, 0) < 0 || !WIFEXITED(st) || WEXITSTATUS(st) != 0) {
            err += "rank " + std::to_string(i + 1) + " failed; ";
            ok = false;
        }
    }
    return ok;
}

bool file_rendezvous(const std::string& path, int rank, uint8_t id[128], double timeout_s, std::string& err) {
    if (rank == 0) {
        const std::string tmp = path + ".tmp";
        FILE* f = std::fopen(tmp.c_str(), "wb");
        if (!f || std::fwrite(id, 1, 128, f) != 128) {
            err = "cannot write " + tmp;
            if (f) std::fclose(f);
            return false;
        }
        std::fclose(f);
        if (std::rename(tmp.c_str(), path.c_str()) != 0) {
            err = "cannot rename " + tmp;
            return false;
        }
        return true;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        FILE* f = std::fopen(path.c_str(), "rb");
        if (f) {
            const size_t k = std::fread(id, 1, 128, f);
            std::fclose(f);
            if (k == 128) return true;
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
            err = "timed out waiting for " + path;
            return false;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
}

}  // namespace skmf
