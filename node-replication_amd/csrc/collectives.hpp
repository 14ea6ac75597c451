// collectives.hpp — the collective calls a replica group makes (group.cpp), as a table of
// function pointers: RCCL's own (resolved with dlopen at the first group call), or the
// in-process loopback of loopback.cpp that tests select with nrg_test_loopback_collectives
// (include/nrgpu_testing.h) to run a G-member group on one GPU.
#pragma once

#include <rccl/rccl.h>

namespace nrg {

struct Collectives {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclSend) send = nullptr;  // partitioned rounds only
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;  // RCCL: unblocks a collective a peer never posted
    void (*set_timeout_ms)(uint32_t) = nullptr;  // loopback: how long this thread's collectives
                                                 // wait for their peers (RCCL: none)
};

// loopback.cpp: every member of a group lives in this process; ncclGroupEnd turns the posted
// all-gathers and send/recv pairs into device copies ordered by events on the members' streams.
const Collectives* loopback_collectives();

}  // namespace nrg
