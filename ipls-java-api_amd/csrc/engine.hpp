// engine.hpp -- the single-device aggregation engine (engine.hip) as the
// multi-device front (ipls_agg.cpp) sees it.  One engine holds the
// accumulators of a contiguous block of the handle's partitions on one GPU;
// engine partition q is handle partition p_lo + q.  Every function has the
// meaning of the C-ABI entry point of the same suffix (include/ipls_agg.h)
// restricted to that block; none of them is exported from the library.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/ipls_agg.h"

struct ipls_dev;
struct ipls_stage;   // the staging one chunked call owns (engine.hip)

const char* dev_last_error(const ipls_dev* h);
void dev_set_thread_error(const char* msg);
// The calling thread's current HIP device, tracked while a C-ABI call runs so
// that switching to a device that is already current costs no HIP call:
// dev_use(d) makes d current (hipSetDevice only when the tracked device
// differs); dev_track(d) records what the thread's device is (-1: unknown,
// every dev_use then sets it); dev_tracked() returns the record.  Every device
// switch on a calling thread goes through dev_use, so the record stays exact.
hipError_t dev_use(int device);
void dev_track(int device);
int dev_tracked();
int dev_geometry(const ipls_agg_cfg* cfg, std::vector<int64_t>& len, std::vector<int64_t>& off, int64_t& chunk,
                 std::string& why);
int dev_open(const ipls_agg_cfg* cfg, int device, int p_lo, int p_hi, ipls_dev** out);
int dev_close(ipls_dev* h);
int dev_device(const ipls_dev* h);
void* dev_stream(ipls_dev* h);
int dev_sync(ipls_dev* h);
int dev_wait(ipls_dev* h, uint64_t ticket);
int dev_flush(ipls_dev* h);
int dev_set_coalesce(ipls_dev* h, int max_group);
int dev_last_launch(const ipls_dev* h, ipls_launch_info* out);

int dev_load_model(ipls_dev* h, const void* src, int64_t n, int src_kind);
int dev_split(ipls_dev* h, const void* flat, int64_t n, int src_kind, int p, void* dst, int dst_kind);
int dev_update_gradient(ipls_dev* h, const void* flat, int64_t n, int src_kind, const int32_t* owned, int n_owned);
int dev_accumulate(ipls_dev* h, int p, int target, const void* src, int64_t n, int src_kind);
int dev_accumulate_async(ipls_dev* h, int p, int target, const void* src, int64_t n, int src_kind, uint64_t* ticket);
int dev_accumulate_range(ipls_dev* h, int p, int target, const void* src, int64_t off, int64_t n, int src_kind,
                         uint64_t* ticket);
int dev_read_range(ipls_dev* h, int p, int target, void* dst, int64_t off, int64_t n, int dst_kind, uint64_t* ticket);
int dev_accumulate_chunked(ipls_dev* h, int p, int target, int64_t n, int src_kind, int64_t chunk,
                           ipls_chunk_source source, void* ctx);
int dev_finalize_chunked(ipls_dev* h, int p, int sum_kind, int64_t chunk, ipls_chunk_sink sink, void* ctx);
int dev_get_partitions_chunked(ipls_dev* h, int64_t chunk, ipls_chunk_sink sink, void* ctx, bool wire);
// the two phases of dev_get_partitions_chunked: the snapshot under the
// engine lock (into a stage the call owns; null for an empty segment), then
// the delivery to the sink with no lock held, which releases the stage
int dev_get_partitions_snapshot(ipls_dev* h, int64_t chunk, bool wire, ipls_stage** st);
int dev_get_partitions_deliver(ipls_dev* h, ipls_stage* st, int64_t chunk, ipls_chunk_sink sink, void* ctx);
void dev_stage_release(ipls_dev* h, ipls_stage* st);
int dev_update_indirect(ipls_dev* h, int p, int target, const void* bytes, int64_t n_bytes);
int dev_gbuf_load(ipls_dev* h, const void* bytes, int64_t n_bytes, const void** gbuf, int64_t* glen);
int dev_other_replica(ipls_dev* h, int p, int32_t aggregator, const void* src, int64_t n, int src_kind);
int dev_other_check(ipls_dev* h);
int dev_other_replica_drop(ipls_dev* h, int p, int32_t aggregator);
// order: n_order engine-local (p, aggregator) pairs, every stored key once
int dev_collect_replicas(ipls_dev* h, int32_t* participants, const int32_t* order, int n_order);
int dev_reduce_batch(ipls_dev* h, int p_first, int n_parts, const void* const* bufs, int k, int src_kind,
                     int start_mode, int target);
int dev_reduce_batch_out(ipls_dev* h, int p_first, int n_parts, const void* const* bufs, int k, int src_kind,
                         int start_mode, void* const* dst, int dst_kind);
int dev_reduce_ext(ipls_dev* h, int n, const int64_t* lens, const void* const* bufs, int k, bool be_in,
                   int start_mode, void* const* dst);
int dev_ingest_pubsub(ipls_dev* h, int target, const uint8_t* const* msgs, const int64_t* lens, int n_msgs,
                      int layers, const int32_t* parts, int32_t* status);
int dev_blend(ipls_dev* h, int p, int target, const void* src, int64_t n, int src_kind, double a, double b);
int dev_scale(ipls_dev* h, int p, int dst_target, int src_target, double c);
int dev_finalize(ipls_dev* h, int p, void* sum_out, int sum_kind, double* avg_out);
int dev_aggregate_round(ipls_dev* h, int p_first, int n_parts, const void* const* bufs, int k, int src_kind,
                        void* avg_out, int avg_kind);
int dev_set_weights(ipls_dev* h, int p, const void* src, int64_t n, int src_kind);
int dev_get_partitions(ipls_dev* h, void* out, int64_t n, int out_kind);
int dev_read(ipls_dev* h, int p, int target, void* dst, int64_t n, int dst_kind);
int dev_promote_future(ipls_dev* h, const int32_t* parts, int n_parts);
int dev_reset(ipls_dev* h, int p);
int dev_device_ptr(ipls_dev* h, int p, int target, void** ptr);
int dev_checksum(ipls_dev* h, int p, int target, uint64_t* out);
int64_t dev_commit_partial(ipls_dev* h, int p, int32_t workers, uint8_t* out, int64_t out_cap);
int64_t dev_merge_files(ipls_dev* h, const uint8_t* const* files, const int64_t* lens, int k, int file_kind,
                        uint8_t* out, int64_t out_cap);
int64_t dev_publish_many(ipls_dev* h, int n, const int* parts, int target, int32_t a, const int32_t* b, int16_t pid,
                         const uint8_t* origin, int32_t origin_len, void* out, const int64_t* offs,
                         const int64_t* lens, int out_kind);
int64_t dev_publish(ipls_dev* h, int p, int target, int32_t a, int32_t b, int16_t pid, const uint8_t* origin,
                    int32_t origin_len, void* out, int64_t out_cap, int out_kind);
