/*
 * framesum — MI355X-native batched frame-checksum engine (C ABI).
 *
 * Drop-in boundary for the soypat/seqs per-frame checksum path. The Go
 * reference computes, for every frame through stacks.PortStack.RecvEth, the
 * RFC 791/1071 one's-complement checksums of eth/crc.go + eth/headers.go one
 * frame per synchronous call. This ABI replaces those per-frame calls with
 * one batched, device-resident call; the per-frame Go functions stay as they
 * are. Plain pointers and sizes only: no HIP, torch or C++
 * types cross the boundary, so cgo / ctypes / JNI can bind it directly
 * (INTEGRATION.md shows the bindings).
 *
 * Replaced reference interfaces (paths relative to the soypat/seqs root):
 *   fs_digest.l4_csum + fs verdict  <- stacks/portstack.go:239-244 (UDP) and
 *        :301-308 (TCP): `gotsum := uhdr.CalculateChecksumIPv4(&ihdr, payload)`
 *        / `thdr.CalculateChecksumIPv4(&ihdr, tcpOptions, payload)` and the
 *        compare that yields ErrChecksumTCPorUDP (portstack.go:132), together
 *        with the RecvEth gates that choose the L4 range (:167-214, :226-237,
 *        :285-299) and the verdict errors (:120-142).
 *   fs_digest.ip_csum               <- eth/headers.go:333-340
 *        (*IPv4Header).CalculateChecksum() applied to frame[14:34].
 *   the CRC791 arithmetic itself    <- eth/crc.go:13-84 (Write/AddUint16/
 *        AddUint32/AddUint8/Sum16/Reset), evaluated on the GPU.
 *   fs_digest.crc32                 <- NEW: IEEE 802.3 CRC-32 (Ethernet FCS)
 *        over frame[0:len). The reference has no CRC-32.
 *
 * Conventions (mirroring the reference's): pure functions over caller-owned
 * buffers, no retention after the call's stream work completes; malformed
 * frames are reported per frame in `status` (the RecvEth error class), never
 * as a call failure. Errors of the call itself are negative fs_status codes
 * (no exceptions cross the ABI); fs_last_error() gives the message.
 * Threading: one fs_ctx per host thread (a context is not internally locked).
 */
#ifndef FRAMESUM_H
#define FRAMESUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FRAMESUM_ABI_VERSION 1u

typedef int32_t fs_status;
#define FS_SUCCESS 0
#define FS_E_INVALID (-1)   /* bad argument (null pointer, n too large, ...) */
#define FS_E_HIP (-2)       /* HIP runtime error (message in fs_last_error) */
#define FS_E_NOMEM (-3)     /* device or pinned-host allocation failed */
#define FS_E_NODEVICE (-4)  /* no such device / device is not gfx950 */

/* Per-frame verdict written to `status` (stacks/portstack.go:120-142). The
 * stack model: MTU `mtu` (0 disables both MTU gates so jumbo frames can be
 * evaluated; the reference caps MTU at 2048, portstack.go:17,46-48), address
 * filters off (MAC :185-186 and IP destination :209-210 are socket-layer
 * policy, not checksum inputs), one UDP and one TCP port open. */
enum fs_verdict {
    FS_OK = 0,                          /* L4 checksum verified (RecvEth continues) */
    FS_ERR_PACKET_SMOL = 1,             /* errPacketSmol */
    FS_ERR_EXCEEDS_MTU = 2,             /* errPacketExceedsMTU */
    FS_IGNORED_NOT_IPV4 = 3,            /* RecvEth returns nil: not IPv4/ARP */
    FS_ARP = 4,                         /* ARP frame (no checksum) */
    FS_ERR_IP_VERSION = 5,              /* errIPVersion */
    FS_ERR_INVALID_IHL = 6,             /* errInvalidIHL */
    FS_ERR_BAD_IP_TOTAL_LEN_OR_IHL = 7, /* errBadIPTotalLenOrIHL */
    FS_ERR_UNKNOWN_IP_PROTO = 8,        /* errUnknownIPProto */
    FS_ERR_TOO_SHORT_TCP_OR_UDP = 9,    /* errTooShortTCPOrUDP */
    FS_ERR_ZERO_PORT = 10,              /* errZeroPort */
    FS_ERR_BAD_UDP_LENGTH = 11,         /* errBadUDPLength */
    FS_ERR_BAD_TCP_OFFSET = 12,         /* errBadTCPOffset */
    FS_ERR_CHECKSUM = 13,               /* ErrChecksumTCPorUDP */
    FS_ERR_FCS = 14                     /* fs_digest_batch_fcs only: FCS missing or wrong (the
                                           frame is dropped before RecvEth; not in the reference) */
};

/* 8-byte per-frame digest. crc32: IEEE CRC-32 of frame[0:len).
 * ip_csum: IPv4Header.CalculateChecksum() of frame[14:34] (0 if len < 34).
 * l4_csum: the TCP/UDP checksum RecvEth computes (`gotsum`), 0 when the frame
 * is rejected before the compare (status not FS_OK / FS_ERR_CHECKSUM). */
typedef struct fs_digest {
    uint32_t crc32;
    uint16_t ip_csum;
    uint16_t l4_csum;
} fs_digest;

typedef struct fs_ctx fs_ctx;

/* Library / device queries. */
uint32_t fs_abi_version(void);
int fs_device_count(void);

/* Context: owns the device copy of the CRC shift tables, a host-mapped report block (the
 * automatic kernel choice), the host-staged entry points' staging buffers and pinned mirrors,
 * and three internal streams for them (a compute stream and two copy streams). */
fs_status fs_ctx_create(int device, fs_ctx** out);
fs_status fs_ctx_destroy(fs_ctx* ctx);
/* Message for the last failing call on `ctx` (or of fs_ctx_create when ctx is NULL). */
const char* fs_last_error(const fs_ctx* ctx);

/* Every batched call takes at most 2^31 frames (n); larger n is FS_E_INVALID. */

/* Batched digest, device-resident. All pointers are DEVICE pointers.
 *   frame i = frames[offsets[i] : offsets[i] + lengths[i]]  (any byte alignment,
 *   frames may overlap or be sparse; the engine reads whole 64-byte-aligned
 *   blocks that hold frame bytes -- up to 63 bytes around a frame, never outside
 *   the memory pages that hold its bytes -- and ignores the bytes outside it).
 *   out[i] receives the digest; status (nullable) receives the fs_verdict.
 * Asynchronous on `stream` (a hipStream_t; NULL = the null stream). */
fs_status fs_digest_batch(fs_ctx* ctx, const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths,
                          uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status, void* stream);

/* TX checksum fill, device-resident and in place. The
 * reference fills a frame's checksums while it builds the frame from header structs:
 *   stacks/port_tcp.go:178 `pkt.IP.Checksum = pkt.IP.CalculateChecksum()` and :193
 *   `pkt.TCP.Checksum = pkt.TCP.CalculateChecksumIPv4(&pkt.IP, nil, payload)`;
 *   stacks/dhcp_client.go:479/:486 and dhcp_server.go:203/:216 (IP, then UDP).
 * For frames whose headers are already in place, flags:
 *   FS_FILL_CSUM  writes the IPv4 header checksum (eth/headers.go:333-340) to frame[24:26]
 *                 and the TCP/UDP checksum RecvEth verifies (the same arithmetic, with the
 *                 frame's own TCP options; none when the data offset is 5, as :193 passes
 *                 nil; frames with options are an extension of the reference's TX path,
 *                 parity unpinned) to the L4 checksum field, both big-endian, for every frame whose
 *                 RecvEth evaluation reaches the checksum compare (verdict FS_OK or
 *                 FS_ERR_CHECKSUM before the fill); other frames are not written.
 *   FS_FCS_APPEND writes the IEEE CRC-32 of the frame (as filled) little-endian at
 *                 frame[len:len+4), the FCS in wire order: those 4 bytes must be spare
 *                 (part of no frame of the batch).
 * out/status receive what fs_digest_batch would report for the frames as written (filled
 * frames: FS_OK). Frames must not overlap. Asynchronous on `stream`. */
#define FS_FILL_CSUM 1u
#define FS_FCS_APPEND 2u
fs_status fs_fill_batch(fs_ctx* ctx, uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                        uint32_t mtu, uint32_t flags, fs_digest* out, uint8_t* status, void* stream);

/* fs_fill_batch from/to HOST memory (the TX buffer a stack writes frames into): copies the
 * batch's byte span to the device, fills, copies the span back into `frames`, and returns
 * when the frames and `out`/`status` are written. frames_bytes bounds every frame (plus its
 * 4 FCS bytes with FS_FCS_APPEND). */
fs_status fs_fill_batch_host(fs_ctx* ctx, uint8_t* frames, uint64_t frames_bytes, const uint64_t* offsets,
                             const uint32_t* lengths, uint32_t n, uint32_t mtu, uint32_t flags, fs_digest* out,
                             uint8_t* status);

/* RX of raw wire frames that still carry their 4-byte FCS (NICs that do not strip it;
 * SURVEY.md §8f rank 4, not in the reference): lengths[i] includes the FCS. out/status are
 * fs_digest_batch's for frame[0:len-4), the bytes RecvEth would receive, except that status
 * is FS_ERR_FCS when len < 4 or the little-endian FCS differs from that CRC-32. */
fs_status fs_digest_batch_fcs(fs_ctx* ctx, const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths,
                              uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status, void* stream);

/* Same computation from/to HOST memory (the NIC / loopback buffer handed to
 * RecvEth): stages H2D, runs the kernel and copies D2H on the context's
 * stream, returning when the results are in `out`/`status`. Pinned memory
 * (fs_host_alloc) gives full PCIe rate; pageable memory works (offsets, lengths, out and status
 * that are pinned are copied straight from / to, or written by the kernel in place, the others go
 * through the context's pinned mirror; an array counts as pinned only when all of it lies inside
 * one pinned allocation). With fs_ctx_set_kernel 0 or 8 a batch whose frames are all <= 128 bytes
 * runs the small-frame kernel: the lengths are on the host here; when its frames, offsets and
 * lengths are all pinned, that kernel reads them in place over PCIe (one launch, no copy). */
fs_status fs_digest_batch_host(fs_ctx* ctx, const uint8_t* frames, uint64_t frames_bytes, const uint64_t* offsets,
                               const uint32_t* lengths, uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status);

/* Multi-GPU form of fs_digest_batch_host for one host process (BASELINE configs[4]: frames
 * streamed from host memory to several GPUs; SURVEY.md §8b fs_digest_batch_multi). Replaces
 * the same per-frame calls as fs_digest_batch_host (stacks/portstack.go:163 RecvEth ->
 * :240 / :303 CalculateChecksumIPv4), for a NIC ring too large for one GPU's PCIe link.
 * The batch is cut into nctx contiguous blocks of frames holding about equal byte counts;
 * block k runs on ctxs[k] (one context per GPU; several contexts may share a GPU), every
 * block at once, each on its own host thread with its own H2D / kernel / D2H pipeline.
 * A block's digests and verdicts are copied straight into out/status at the block's own
 * indices: the host arrays are the gather, so no device collective is involved (the
 * device-resident RCCL form is fs_digest_batch_sharded below).
 * Blocks are runs of frames in BUFFER order: when the offsets are not non-decreasing, the
 * frames are first ordered by offset, so each context still copies only its own bytes.
 * ctxs must be distinct. Returns when every block is done; on failure, the status of the
 * lowest failing block, whose message is in fs_last_error of that block's context (every
 * entry point clears its context's message first, so only failing contexts hold one). */
fs_status fs_digest_batch_multi(fs_ctx* const* ctxs, int nctx, const uint8_t* frames, uint64_t frames_bytes,
                                const uint64_t* offsets, const uint32_t* lengths, uint32_t n, uint32_t mtu,
                                fs_digest* out, uint8_t* status);

/* ---- Device-resident multi-GPU form with RCCL (BASELINE configs[3], C4; SURVEY.md §8b
 * "N GPUs + RCCL gather", §8e). Replaces the same per-frame calls as fs_digest_batch
 * (stacks/portstack.go:163 RecvEth -> :240 / :303 CalculateChecksumIPv4) for a batch held
 * in the HBM of several GPUs of one node, driven from ONE host process (a Go PortStack):
 * frames are independent (eth/crc.go:12-17, CRC791 is per call), so the batch shards with
 * no data-path collective, and RCCL over xGMI is used only to gather the 8-byte digests and
 * 1-byte verdicts back to the first device.
 *
 * A group holds one context, one stream and one RCCL communicator (ncclCommInitAll) per
 * device; devices must be distinct. */
typedef struct fs_group fs_group;
fs_status fs_group_create(const int* devices, int ndev, fs_group** out);
fs_status fs_group_destroy(fs_group* g);
/* Message for the last failing call on `g` (or of fs_group_create when g is NULL). */
const char* fs_group_last_error(const fs_group* g);

/* Round-robin sharding of a global batch of n frames over nshards shards: global frame i
 * is local frame i / nshards of shard i % nshards; shard k holds fs_shard_count(n, nshards, k)
 * frames. */
uint64_t fs_shard_count(uint64_t n, uint32_t nshards, uint32_t shard);

/* Digest a global batch sharded round-robin over the group's devices. frames[k], offsets[k],
 * lengths[k] are DEVICE pointers on the group's k-th device describing shard k (its
 * fs_shard_count(n, ndev, k) frames, laid out as fs_digest_batch expects). The call works in
 * chunks of the shards' rows (at most 8, ~32K rows each). For each chunk, every device digests
 * its rows on its own compute stream; its digest and verdict pieces then go to the first
 * device by grouped point-to-point RCCL transfers (ncclSend / ncclRecv on a second stream per
 * device), and a de-interleave kernel there puts that chunk's frames in global order. So a
 * chunk's transfer and de-interleave overlap the next chunk's kernels. out (n digests) and
 * status (n bytes, nullable) are DEVICE pointers on the group's first device. Returns when
 * they are written; on an error return every stream of the group has been drained first, so
 * no work of the failed call is still in flight. At most 2^31 frames per shard. N > 1
 * devices has not run on hardware (the build boxes have one GPU). */
fs_status fs_digest_batch_sharded(fs_group* g, const uint8_t* const* frames, const uint64_t* const* offsets,
                                  const uint32_t* const* lengths, uint64_t n, uint32_t mtu, fs_digest* out,
                                  uint8_t* status);

/* The de-interleave step alone, for callers that gather the shards themselves (one process
 * per GPU, e.g. torch.distributed over RCCL): `gathered` (device memory of ctx's device)
 * holds nshards slabs back to back; slab k is shard k's m = ceil(n / nshards) digests (8 B
 * each) followed by its m verdict bytes, padded to a multiple of 256 bytes:
 * fs_shard_slab_bytes(n, nshards) bytes per slab. Writes out[i] / status[i] (nullable) for
 * global frames i < n. Asynchronous on `stream`. */
uint64_t fs_shard_slab_bytes(uint64_t n, uint32_t nshards);
fs_status fs_deinterleave(fs_ctx* ctx, const uint8_t* gathered, uint32_t nshards, uint64_t n, fs_digest* out,
                          uint8_t* status, void* stream);

/* Kernel variant of a context's launches. The engine has four kernels: a one-pass kernel for
 * batches of similar frame lengths (each frame read as the 64-byte blocks that hold it), a
 * mixed-length kernel that splits long frames into 768-byte pieces when a tile of 16 frames mixes
 * very different lengths, a segment kernel that cuts every frame of such a tile into equal chunks
 * (for tiles whose longest frame is beyond the pieces' reach, e.g. a 128-KB frame among 64-byte
 * ones), and a small-frame kernel (one lane per frame, small workgroups) for traffic of short
 * frames such as the reference's 47-byte benchmark frames. The kernels report whether a launch's
 * batch had mixed-length tiles (and whether one of them held such a giant frame) and whether it had
 * a frame longer than 128 bytes (sampled on steady traffic: each report is a store to host memory);
 * the host reads those reports a few launches late.
 *   0 (default): automatic. Mixed-length tiles select the mixed-length kernel (the segment kernel
 *     when the report says giant), similar lengths the one-pass kernel; after 16 launches seen to
 *     run with no frame over 128 bytes, the small-frame kernel, until a launch reports a longer frame.
 *   2 / 3 / 4: always the mixed-length / the segment / the one-pass kernel.
 *   8: the small-frame kernel preferred: it runs until a launch reports a frame over 128 bytes,
 *     then the automatic choice among the others until 2 launches have run short again.
 * The host-staged calls see every length: with 0 or 8 a batch whose frames are all <= 128 bytes
 * runs the small-frame kernel; with 0 a batch whose lengths all lie within 256 bytes of each other
 * runs the one-pass kernel from the context's first call; any other batch the automatic choice. A
 * TX fill never runs the small-frame kernel. Because reports arrive late, a launch of the
 * small-frame kernel can still meet long frames: they stay correct there but one lane streams each
 * of them (hundreds of us for a batch of jumbo frames). Any other variant is FS_E_INVALID. Results
 * are identical in every case; only the speed differs. */
fs_status fs_ctx_set_kernel(fs_ctx* ctx, int variant);

/* The kernel (2 mixed-length, 3 segment, 4 one-pass, 8 small-frame) the context's latest launch
 * ran; 0 before its first launch, FS_E_INVALID for a null context. With variant 0 a context's first
 * 16 device-resident launches run the mixed-length kernel (2), which keeps itself chosen while it
 * meets mixed tiles (moving to the segment kernel, 3, when they hold giant frames); uniform traffic
 * then moves to the one-pass kernel (4), and traffic of frames <= 128 bytes to the small-frame
 * kernel (8). The window costs uniform 1500-byte traffic about 1.5 us per launch (~23 us once per
 * context, measured on MI355X); mixed traffic it saves ~80 us per launch. A caller that knows its
 * device-resident traffic is uniform can set variant 4 (host-staged calls see the lengths and skip
 * the window for uniform batches by themselves). */
int fs_ctx_last_kernel(const fs_ctx* ctx);

/* Workgroups per launch of a context's kernels: 0 (the default) launches one 16-wave
 * workgroup per compute unit, so a batch of 65,536 frames gives every wave one tile of 16
 * frames; k > 0 caps the grid at k workgroups (at most one per CU), so each wave streams
 * several tiles back to back and consecutive launches on other streams run side by side on
 * the remaining CUs. A negative value is FS_E_INVALID. Results never depend on it. */
fs_status fs_ctx_set_workgroups(fs_ctx* ctx, int workgroups);

/* Pinned host memory helpers for fs_digest_batch_host callers. */
fs_status fs_host_alloc(fs_ctx* ctx, uint64_t bytes, void** out);
fs_status fs_host_free(fs_ctx* ctx, void* p);

#ifdef __cplusplus
}
#endif
#endif /* FRAMESUM_H */
