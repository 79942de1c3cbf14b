// In-graph event nodes for the overlapped gradient all-reduce (visionseg/optim.py
// GradReducer): while the forward+backward step is captured into a HIP graph, each
// all-reduce bucket's completion point is marked with an EXTERNAL event record
// (hipEventRecordWithFlags(..., hipEventRecordExternal)), which the capture turns into an
// event-record node of the graph instead of a capture-internal dependency.  After the
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
  VS_HIP(hipEventRecordWithFlags((hipEvent_t)event, (hipStream_t)stream, hipEventRecordExternal));
  return VS_OK;
}

extern "C" int vs_stream_wait_event(void* stream, void* event) {
  VS_CHECK(event, "null event");
  VS_HIP(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
  return VS_OK;
}
