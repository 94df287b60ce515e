// skm_mesh.h -- process-per-rank launch for the drop-in CLIs and a host transport over a full
// mesh of socketpairs (skm_transport, include/skm.h).  Plain C++ (POSIX), no HIP.
//
// mesh_fork(W) forks W-1 children before any GPU or thread use; rank 0 stays in the caller.
// Every process pair is joined by a socketpair (host transport: --comm host) and every child by
// a pipe from rank 0 (the RCCL unique id: --comm rccl).
#pragma once

#include <sys/types.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "skm.h"

namespace skmf {

struct Mesh {
    int rank = 0, world = 1;
    std::vector<int> fd;            // socket to peer q (-1: self)
    int id_pipe = -1;               // children: read end of the unique-id pipe from rank 0
    std::vector<int> id_pipes;      // rank 0: write ends, [q] for child q
    std::vector<pid_t> children;    // rank 0: child pids, [q - 1] for rank q
    skm_transport transport();      // ctx = this
    // RCCL unique id from rank 0 to every child (rank 0 passes the id it made)
    bool share_id(uint8_t id[128], std::string& err);
    // rank 0: wait for every child; false (with err) if any failed
    bool wait_children(std::string& err);
    // rank 0: until wait_children, a thread polls the children; one that fails makes rank 0
    // terminate the others and exit 1 (a rank blocked in an RCCL collective would wait forever).
    // Children die with rank 0 (PR_SET_PDEATHSIG).
    void watch_children();
    std::shared_ptr<std::atomic<bool>> watching;
};

// fork world-1 children; returns false on failure (err set).  In each process m.rank is its rank.
bool mesh_fork(int world, Mesh& m, std::string& err);

// external launcher (RANK / WORLD_SIZE / LOCAL_RANK in the environment): the RCCL unique id
// through a file rank 0 writes (atomic rename) and the others poll for (up to timeout_s)
bool file_rendezvous(const std::string& path, int rank, uint8_t id[128], double timeout_s, std::string& err);

}  // namespace skmf
