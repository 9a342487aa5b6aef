// Stream-capture topology guard.
//
// Root cause of the round-4 crash (profiles/r4/sdma_split_attempt.log, reproduced by tools/probes/capture_probe3.hip,
// profiles/r5/capture/): HIP 7.2's hipStreamEndCapture faults (SIGSEGV inside the runtime) when, inside one capture, a
// stream forked from a NON-origin stream waits on an event recorded by its sibling — the round-4 split: per slab face
// two copy streams forked from the exchange stream, the signal stream waiting for the other copy stream. Run eagerly
// the same schedule is fine; adding a direct join of the sibling into the parent does not help (probe mode 5); the
// production topologies (one copy stream per face or per message group, every copy stream forked from and joined into
// the exchange stream, which forks from and joins into s0: modes 0, 1) and joins through the parent (modes 3, 4) capture
// and replay. Streams forked from the capture's origin waiting on each other (a group's per-rank s0 / s1) are fine.
//
// Every cross-stream dependency of a captured schedule goes through record() / wait(): the guard keeps the fork tree of
// the capture (thread-local, like hipStreamCaptureModeThreadLocal; a stream's parent = the stream whose event it first
// waited on) and refuses the crashing wait with a message BEFORE it enters the capture. close() then joins every stream
// of the aborted capture into its parent, deepest first, so hipStreamEndCapture sees a joined graph.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace wave3d::capture {

void begin(hipStream_t origin);            // after hipStreamBeginCapture(origin)
void record(hipEvent_t e, hipStream_t s);  // hipEventRecord(e, s) + bookkeeping while a capture is active
void wait(hipStream_t s, hipEvent_t e);    // hipStreamWaitEvent(s, e, 0); throws (fail) on the crashing topology
void finish();                             // the schedule is enqueued: stop tracking
void close();                              // an aborted capture: join every stream into its parent, stop tracking
void abandon();                            // after hipStreamEndCapture: release close()'s events, forget the state
bool active();

// the probe topologies through the guard, captured and launched on the current device (tests): mode 0 = one copy
// stream per face (production), 2 = the round-4 split. Returns "ok" or the refusal message.
std::string selftest(int mode);

}  // namespace wave3d::capture
