// In-graph event nodes for the overlapped gradient all-reduce (visionseg/optim.py
// GradReducer): while the forward+backward step is captured into a HIP graph, each
// all-reduce bucket's completion point is marked with an EXTERNAL event record
// (an event-record node added to the graph being captured, after the stream's capture
// frontier) instead of a capture-internal dependency.  After the
// graph is launched, a side stream waits on those events (hipStreamWaitEvent) and issues
// the RCCL all-reduce of each bucket there, overlapping the rest of the replay.
// (torch.cuda.Event(external=True) is refused on ROCm builds of PyTorch, hence these
// four entry points.)
#include "common.h"

using namespace vs;

extern "C" int vs_event_create(void** event) {
  VS_CHECK(event, "null pointer");
  hipEvent_t e;
  VS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  *event = (void*)e;
  return VS_OK;
}

extern "C" int vs_event_destroy(void* event) {
  if (event) VS_HIP(hipEventDestroy((hipEvent_t)event));
  return VS_OK;
}

extern "C" int vs_event_record_external(void* event, void* stream) {
  VS_CHECK(event, "null event");
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t e = (hipEvent_t)event;
  hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  VS_HIP(hipStreamGetCaptureInfo_v2(s, &status, &id, &graph, &deps, &ndeps));
  if (status != hipStreamCaptureStatusActive) {
    VS_HIP(hipEventRecord(e, s));
    return VS_OK;
  }
  // Under capture: what hipEventRecordWithFlags(..., hipEventRecordExternal) documents
  // (the ROCm 7.2 runtime rejects that flag during capture), done by hand: an
  // event-record node after the stream's current capture frontier, which then becomes
  // the frontier.
  hipGraphNode_t node;
  VS_HIP(hipGraphAddEventRecordNode(&node, graph, deps, ndeps, e));
  VS_HIP(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
  return VS_OK;
}

extern "C" int vs_stream_wait_event(void* stream, void* event) {
  VS_CHECK(event, "null event");
  VS_HIP(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
  return VS_OK;
}
