// mppi_aql.h -- native dispatch of the control step (mppi_aql.cpp).  Internal.
//
// mppi_run_steps' (rollout, finalize) pairs as raw AQL kernel-dispatch packets on an HSA
// queue the engine owns, instead of one hipLaunchKernel per kernel: the kernels come from
// the library's own gfx950 code objects (lib/<library>.<unit>.co, loaded through the HSA
// loader), their argument blocks live in device memory and are written only when their
// content changes.  The rollout's Philox step counter -- the one argument that changes every
// step -- is passed relative to the dispatch id (the packet's index in the queue, which the
// waves receive in SGPRs): step = arg + (id >> 1), the queue holding (rollout, finalize)
// pairs only.  The host's work per step is two 64 B packets and a doorbell store.
#pragma once
#include <stdint.h>

#include <mutex>
#include <string>

#include "mppi_dev.h"

namespace mppi_aql {

struct Step;   // one engine's queue, completion signal and device-resident argument blocks

// nullptr (and why) when native dispatch is unavailable on this device ordinal.
// The queue is probed first (two packets report their dispatch ids): a queue whose dispatch ids
// are not its packet indices (intercepted by a tool) is refused.
Step* step_create(int device, std::string* why);
// false: the queue did not drain (60 s); it is inactivated and its memory leaked, and the caller
// must not free buffers its kernels may still use.
bool step_destroy(Step* s);

// Make the device-resident argument blocks hold these two launches such that the next
// rollout dispatched runs step `step`: the rollout's step word (byte offset step_off of its
// arguments, dispatch-id relative) becomes step - (next packet index >> 1).  Uploads only when
// a launch differs from the resident one (the step word excluded) or the resident step word
// would not give `step`; waits for the queue to drain before overwriting.  0; -2 when the launches
// cannot be dispatched natively (a symbol the code objects lack, hidden arguments);
// -1 on a runtime failure (*err says why).
int step_prepare(Step* s, const mppi::LaunchDesc& roll, const mppi::LaunchDesc& fin, uint32_t step,
                 uint32_t step_off, std::string* err);
// n (rollout, finalize) pairs, each kernel dependent on the one before; the last finalize
// carries the completion signal and a system-scope release.
// overlap: every rollout after the first without the barrier bit (it starts while the finalize
// before it runs and waits for it in the kernel: mppi_device.h kNoiseOverlap)
int step_dispatch(Step* s, int n, std::string* err, bool overlap = false);
// The queue held against other threads' packets (the prewarm thread's step_touch) while the
// guard lives: a step_prepare and the step_dispatch after it must see the same packet index,
// or the batch's rollouts would run later steps than prepared.
std::unique_lock<std::recursive_mutex> step_guard(Step* s);
// One control call: a (rollout, finalize) pair whose rollout arguments (the state changes every
// call) are written by the host into a fresh block of a small ring in host-writable device
// memory (pinned host memory without one), the finalize's from a static device block.  The host
// writes `seq` into the rollout's arguments at seq_off (the vehicle constants' spare word,
// which the rollout hands to the finalize) and polls the completion flags for it: bit 31 set,
// unique per call.  0 / -2 / -1 as step_prepare.
int step_call(Step* s, const mppi::LaunchDesc& roll, const mppi::LaunchDesc& fin, uint32_t step,
              uint32_t step_off, uint32_t seq_off, uint32_t* seq, std::string* err);
// The last call's outputs have been seen (its completion flags): its rollout has run.
void step_call_read(Step* s);
// Where the control calls' rollout arguments live ("device kernarg pool", "device
// fine-grained", "device coarse-grained": written by the host through the BAR; or "pinned host
// memory", read over PCIe by every block: MPPI_AQL_CALL_HOSTMEM=1 or no host-writable pool).
const char* step_call_memory(Step* s);
// Two one-wave packets (k_dispatch_probe into a scratch word) on the engine's queue: its
// packet processor and queue state exercised, no engine buffer touched (the next batch re-uploads
// its step word: the pair moved the packet indices).  From any thread.  if_free: 1 without
// touching when another thread holds the queue.  0 / 1 / -1 (a queue error).
int step_touch(Step* s, bool if_free, std::string* err);
// The doorbell rung again with the last packet's index: no packet, nothing dispatched.
// Only from the thread that writes the packets (a stale index rung after a newer one would hide
// the newer packets from the packet processor).
void step_ring(Step* s);
// The queue's asynchronous error, if any (0 = none).
int step_error(Step* s);
// Until every dispatched pair has completed.  -1 on a queue error or after timeout_ms.
int step_wait(Step* s, int timeout_ms, std::string* err);
bool step_busy(Step* s);

// Install (or, with nullptr, remove) the calling thread's capture target: the launchers then
// describe their launch into it instead of launching (mppi_device.h go()).
void set_capture(mppi::LaunchDesc* d);

}  // namespace mppi_aql
