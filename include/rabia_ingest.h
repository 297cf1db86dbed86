/*
 * rabia_ingest.h — C ABI of device-side vote ingestion.
 *
 * Turns received wire messages into the packed vote planes the phase step reads
 * (rabia_gpu.h "Layout"). A message is the payload of one TCP MessageFrame
 * (rabia-engine/src/network/tcp.rs:114-176: u32 LE length + payload) =
 * bincode 1.3.3 of ProtocolMessage (rabia-core/src/messages.rs:7-13, 59-94):
 *   id Uuid | from NodeId | to Option<NodeId> | timestamp u64 | MessageType
 * with Uuid (uuid 1.18.0, serde, non-human-readable) = u64 length 16 + 16 bytes,
 * PhaseId/NodeId/BatchId newtypes transparent, enum variants as u32, Option as a
 * u8 tag, HashMap as u64 count + entries, little-endian fixed-width integers.
 *
 * What is recorded, following RabiaEngine::handle_message (engine.rs:350-368) and
 * the vote handlers (engine.rs:483-492, 613-622):
 *  - only VoteRound1 (variant 1) and VoteRound2 (variant 2) change planes; other
 *    variants are counted and skipped;
 *  - ProtocolMessage::validate (rabia-core/src/validation.rs:30-81): timestamp
 *    within [now_ms - 600000, now_ms + 60000]; a VoteRound2 must carry a non-empty
 *    round1_votes map;
 *  - message.from must equal the transport sender (engine.rs:357-364) when
 *    sender_lane is given, and must be a cluster member (lane = its position in
 *    `members`);
 *  - the vote is stored under the SENDER (phase.add_round{1,2}_vote(from, vote)),
 *    not voter_id; last write wins per (round, sender, phase) in message order
 *    (messages.rs:169-175: HashMap::insert), across calls too (planes accumulate);
 *  - a message that bincode::deserialize would reject (short, bad variant, Uuid
 *    length != 16, Option tag > 1, StateValue > 2) is dropped (tcp.rs:583-596).
 * PhaseIds outside [slot_base, slot_base + n_slots) are counted, not recorded.
 *
 * A fresh window's planes must hold "absent" (all bits 1: memset 0xFF).
 * Conventions as rabia_gpu.h (RG_OK or negative rg_status, void* streams, no CPU
 * fallback).
 */
#ifndef RABIA_INGEST_H
#define RABIA_INGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rg_ingest rg_ingest;

typedef struct rg_ingest_config {
  uint32_t n_replicas;    /* lanes, 1..16                                             */
  uint32_t tile_words;    /* plane layout of the vote buffers (0 = planar)            */
  int32_t device;
  uint32_t reserved;
  uint8_t members[16][16]; /* NodeId UUID bytes in lane order (sorted membership)       */
} rg_ingest_config;

/* stats_dev[RG_INGEST_STATS] counters, accumulated over calls (caller zeroes them). */
enum {
  RG_INGEST_R1 = 0,        /* VoteRound1 votes recorded                                */
  RG_INGEST_R2 = 1,        /* VoteRound2 votes recorded                                */
  RG_INGEST_SUPERSEDED = 2,/* valid votes overwritten by a later one in the same call  */
  RG_INGEST_OTHER = 3,     /* non-vote message types                                   */
  RG_INGEST_OUTSIDE = 4,   /* valid votes for PhaseIds outside the window              */
  RG_INGEST_INVALID = 5,   /* rejected by validate() (timestamp, empty round1_votes)   */
  RG_INGEST_SENDER = 6,    /* message.from != sender, or not a member                  */
  RG_INGEST_MALFORMED = 7, /* bincode would not deserialize it                         */
  RG_INGEST_STATS = 8
};

int rg_ingest_create(rg_ingest** out, const rg_ingest_config* cfg);
int rg_ingest_destroy(rg_ingest* ing);
const char* rg_ingest_last_error(const rg_ingest* ing);

/* Record the votes of n_msgs messages (message m = msgs_dev[msg_off_dev[m] ..
 * msg_off_dev[m+1])) into votes_dev (the window's 4n+1 planes). sender_lane_dev
 * (may be NULL) = lane of the connection each message arrived on. */
int rg_ingest_votes_async(rg_ingest* ing, const uint8_t* msgs_dev, const uint64_t* msg_off_dev,
                          const uint8_t* sender_lane_dev, uint64_t n_msgs, uint64_t now_ms,
                          uint32_t* votes_dev, uint64_t n_slots, uint64_t stride_words,
                          uint64_t slot_base, uint64_t* stats_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RABIA_INGEST_H */
