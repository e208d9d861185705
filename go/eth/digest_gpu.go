//go:build framesum

// Package eth addition: the batched, GPU-side form of the checksum work that
// stacks.PortStack.RecvEth and the TX header builders do one frame at a time.
//
// Drop this file into soypat/seqs/eth/ and build with `-tags framesum` next to
// libframesum.so (include/framesum.h of the framesum engine). The existing
// per-frame functions -- CRC791 (crc.go:13-84), (*IPv4Header).CalculateChecksum
// (headers.go:333), (*UDPHeader).CalculateChecksumIPv4 (:382) and
// (*TCPHeader).CalculateChecksumIPv4 (:510) -- stay untouched and remain the
// parity reference: for every frame, DigestBatch returns exactly the L4 checksum
// RecvEth computes (`gotsum`, stacks/portstack.go:239 / :303), the IPv4 header
// checksum of frame[14:34], the IEEE 802.3 CRC-32 of the frame, and the error
// class RecvEth would return (Verdict).
//
// Not compiled in the framesum repository (its build image has no Go toolchain);
// tests/csrc/go_binding_replay.c replays DigestBatch's packing and calls through
// the same C ABI on the GPU and is checked against the CPU oracle.
package eth

/*
#cgo CFLAGS: -I${SRCDIR}/../third_party/framesum/include
#cgo LDFLAGS: -L${SRCDIR}/../third_party/framesum/lib -lframesum -Wl,-rpath,${SRCDIR}/../third_party/framesum/lib
#include <framesum.h>
#include <stdlib.h>
*/
import "C"

import (
	"errors"
	"unsafe"
)

// Digest is the per-frame result of DigestBatch. Its layout is C struct fs_digest.
type Digest struct {
	CRC32  uint32 // IEEE 802.3 CRC-32 of frame[0:len)
	IPCsum uint16 // (*IPv4Header).CalculateChecksum() of frame[14:34]; 0 if the frame is shorter
	L4Csum uint16 // the TCP/UDP checksum RecvEth computes; 0 when RecvEth rejects the frame earlier
}

// Verdict is the error class RecvEth returns for a frame (enum fs_verdict), under the
// engine's stack model: MTU as passed, no MAC / IP destination filter, sockets open for
// both protocols. stacks.PortStack.RecvEthBatch applies the remaining policy.
type Verdict uint8

const (
	VerdictOK                 Verdict = 0  // checksum verified
	VerdictPacketSmol         Verdict = 1  // errPacketSmol
	VerdictExceedsMTU         Verdict = 2  // errPacketExceedsMTU
	VerdictNotIPv4            Verdict = 3  // ignored: neither IPv4 nor ARP
	VerdictARP                Verdict = 4  // ARP frame
	VerdictIPVersion          Verdict = 5  // errIPVersion
	VerdictInvalidIHL         Verdict = 6  // errInvalidIHL
	VerdictBadIPTotalLenOrIHL Verdict = 7  // errBadIPTotalLenOrIHL
	VerdictUnknownIPProto     Verdict = 8  // errUnknownIPProto
	VerdictTooShortTCPOrUDP   Verdict = 9  // errTooShortTCPOrUDP
	VerdictZeroPort           Verdict = 10 // errZeroPort
	VerdictBadUDPLength       Verdict = 11 // errBadUDPLength
	VerdictBadTCPOffset       Verdict = 12 // errBadTCPOffset
	VerdictChecksum           Verdict = 13 // ErrChecksumTCPorUDP
	VerdictFCS                Verdict = 14 // DigestBatchFCS only: FCS missing or wrong
)

// The C struct and this one must agree byte for byte (8 bytes, no padding).
var _ [8]byte = [unsafe.Sizeof(Digest{})]byte{}

// GPU is one framesum context on one device: device CRC tables, staging buffers and
// pinned memory for the frames. Like PortStack, it is not safe for concurrent use.
type GPU struct {
	ctx  *C.fs_ctx
	pin  unsafe.Pointer // pinned staging buffer (fs_host_alloc)
	pcap int
	offs []uint64
	lens []uint32
}

// OpenGPU creates a context on HIP device `device` (an MI355X, gfx950).
func OpenGPU(device int) (*GPU, error) {
	var ctx *C.fs_ctx
	if st := C.fs_ctx_create(C.int(device), &ctx); st != C.FS_SUCCESS {
		return nil, errors.New("framesum: " + C.GoString(C.fs_last_error(nil)))
	}
	return &GPU{ctx: ctx}, nil
}

// Close releases the context and its pinned staging memory.
func (g *GPU) Close() error {
	if g.ctx == nil {
		return nil
	}
	if g.pin != nil {
		C.fs_host_free(g.ctx, g.pin)
		g.pin, g.pcap = nil, 0
	}
	C.fs_ctx_destroy(g.ctx)
	g.ctx = nil
	return nil
}

func (g *GPU) lastErr() error { return errors.New("framesum: " + C.GoString(C.fs_last_error(g.ctx))) }

// Kernel variants of fs_ctx_set_kernel (include/framesum.h): results never depend on them.
const (
	KernelAuto     = 0 // one-pass kernel for uniform lengths, piece-splitting (or segment) kernel for mixed ones, the
	// one-lane-per-frame kernel once the launches seen have had no frame over 128 B;
	// DigestBatch picks the one-lane-per-frame kernel itself for a batch of frames all <= 128 B
	KernelMixed    = 2 // piece-splitting kernel
	KernelSegments = 3 // equal chunks per frame: tiles that mix a giant frame (beyond the pieces) with short ones
	KernelOnePass  = 4 // one-pass kernel
	KernelSmall    = 8 // one lane per frame preferred, until a launch reports a frame over 128 B: a
	// stack whose traffic is short frames (ACKs, DNS, DHCP, the reference's 47-byte benchmark
	// frames in stacks/benchmark_test.go)
)

// SetKernel selects the kernel variant of this context's launches (fs_ctx_set_kernel).
func (g *GPU) SetKernel(variant int) error {
	if st := C.fs_ctx_set_kernel(g.ctx, C.int(variant)); st != C.FS_SUCCESS {
		return g.lastErr()
	}
	return nil
}

// stage packs frames back to back, each at a 4-byte aligned offset, into pinned memory,
// followed by 16 spare bytes (slack for the dword-rounded copy span; on the device the engine
// reads the 64-byte blocks around each frame inside its own staging buffer). The frames'
// offsets and lengths go into the same pinned allocation, after the frames, so that
// fs_digest_batch_host copies them to the device straight from there (no mirror copy on the
// host; DESIGN.md §5.3), and a batch of short frames (all <= 128 B, the reference's benchmark
// shape) is read in place over PCIe by the small-frame kernel: one launch, no copy.
func (g *GPU) stage(frames [][]byte, spare int) ([]byte, error) {
	n := len(frames)
	total := 0
	for _, f := range frames {
		total += (len(f) + spare + 3) &^ 3
	}
	total += 16
	desc := (total + 7) &^ 7 // the descriptors, 8-byte aligned, after the frames
	need := desc + 12*n
	if need > g.pcap {
		if g.pin != nil {
			C.fs_host_free(g.ctx, g.pin)
			g.pin, g.pcap = nil, 0
		}
		var p unsafe.Pointer
		if st := C.fs_host_alloc(g.ctx, C.uint64_t(need), &p); st != C.FS_SUCCESS {
			return nil, g.lastErr()
		}
		g.pin, g.pcap = p, need
	}
	mem := unsafe.Slice((*byte)(g.pin), need)
	g.offs, g.lens = nil, nil
	if n > 0 {
		g.offs = unsafe.Slice((*uint64)(unsafe.Pointer(&mem[desc])), n)
		g.lens = unsafe.Slice((*uint32)(unsafe.Pointer(&mem[desc+8*n])), n)
	}
	buf := mem[:total]
	pos := 0
	for i, f := range frames {
		g.offs[i] = uint64(pos)
		g.lens[i] = uint32(len(f))
		copy(buf[pos:], f)
		pos += (len(f) + spare + 3) &^ 3
	}
	return buf, nil
}

// DigestBatch computes, for every frame, the digest and the RecvEth verdict (mtu as
// PortStack's MTU; 0 disables the MTU gates). out and verdicts must hold len(frames).
func (g *GPU) DigestBatch(frames [][]byte, mtu uint16, out []Digest, verdicts []Verdict) error {
	n := len(frames)
	if len(out) < n || len(verdicts) < n {
		return errors.New("framesum: output slices too short")
	}
	if n == 0 {
		return nil
	}
	buf, err := g.stage(frames, 0)
	if err != nil {
		return err
	}
	st := C.fs_digest_batch_host(g.ctx, (*C.uint8_t)(unsafe.Pointer(&buf[0])), C.uint64_t(len(buf)),
		(*C.uint64_t)(unsafe.Pointer(&g.offs[0])), (*C.uint32_t)(unsafe.Pointer(&g.lens[0])),
		C.uint32_t(n), C.uint32_t(mtu), (*C.fs_digest)(unsafe.Pointer(&out[0])),
		(*C.uint8_t)(unsafe.Pointer(&verdicts[0])))
	if st != C.FS_SUCCESS {
		return g.lastErr()
	}
	return nil
}

// FillBatch is the checksum part of the TX header builders for many frames at once
// (stacks/port_tcp.go:178, :193; dhcp_client.go:479, :486): it writes the IPv4 header
// checksum and the TCP/UDP checksum into every frame RecvEth would checksum, in place
// in frames, and with appendFCS the CRC-32 little-endian after each frame (each frame
// slice must then have 4 bytes of capacity past its length). out / verdicts receive
// what DigestBatch reports for the frames as written.
func (g *GPU) FillBatch(frames [][]byte, mtu uint16, appendFCS bool, out []Digest, verdicts []Verdict) error {
	n := len(frames)
	if len(out) < n || len(verdicts) < n {
		return errors.New("framesum: output slices too short")
	}
	if n == 0 {
		return nil
	}
	spare, flags := 0, C.uint32_t(C.FS_FILL_CSUM)
	if appendFCS {
		spare, flags = 4, flags|C.FS_FCS_APPEND
		for _, f := range frames {
			if cap(f)-len(f) < 4 {
				return errors.New("framesum: FillBatch with appendFCS needs 4 bytes of capacity past each frame")
			}
		}
	}
	buf, err := g.stage(frames, spare)
	if err != nil {
		return err
	}
	st := C.fs_fill_batch_host(g.ctx, (*C.uint8_t)(unsafe.Pointer(&buf[0])), C.uint64_t(len(buf)),
		(*C.uint64_t)(unsafe.Pointer(&g.offs[0])), (*C.uint32_t)(unsafe.Pointer(&g.lens[0])),
		C.uint32_t(n), C.uint32_t(mtu), flags, (*C.fs_digest)(unsafe.Pointer(&out[0])),
		(*C.uint8_t)(unsafe.Pointer(&verdicts[0])))
	if st != C.FS_SUCCESS {
		return g.lastErr()
	}
	for i, f := range frames {
		copy(f[:len(f)+spare], buf[g.offs[i]:g.offs[i]+uint64(len(f)+spare)])
	}
	return nil
}

// GPUs is one host process's set of contexts, one per GPU, for NIC rings larger than one
// PCIe link carries (fs_digest_batch_multi; BASELINE configs[4]).
type GPUs struct {
	gpus []*GPU
	ctxs unsafe.Pointer // C array of fs_ctx* (cgo: Go memory may not hold C pointers passed to C)
	buf  *GPU           // stages the frames (its pinned buffer)
}

// OpenGPUs opens one context per listed device.
func OpenGPUs(devices []int) (*GPUs, error) {
	if len(devices) == 0 {
		return nil, errors.New("framesum: no devices")
	}
	m := &GPUs{ctxs: C.malloc(C.size_t(len(devices)) * C.size_t(unsafe.Sizeof(uintptr(0))))}
	arr := unsafe.Slice((**C.fs_ctx)(m.ctxs), len(devices))
	for i, d := range devices {
		g, err := OpenGPU(d)
		if err != nil {
			m.Close()
			return nil, err
		}
		m.gpus = append(m.gpus, g)
		arr[i] = g.ctx
	}
	m.buf = m.gpus[0]
	return m, nil
}

// Close releases every context.
func (m *GPUs) Close() error {
	for _, g := range m.gpus {
		g.Close()
	}
	m.gpus = nil
	if m.ctxs != nil {
		C.free(m.ctxs)
		m.ctxs = nil
	}
	return nil
}

// DigestBatch spreads the batch over the contexts: byte-balanced runs of frames, each on
// its own GPU, PCIe link and host thread; results in batch order.
func (m *GPUs) DigestBatch(frames [][]byte, mtu uint16, out []Digest, verdicts []Verdict) error {
	n := len(frames)
	if len(out) < n || len(verdicts) < n {
		return errors.New("framesum: output slices too short")
	}
	if n == 0 {
		return nil
	}
	buf, err := m.buf.stage(frames, 0)
	if err != nil {
		return err
	}
	g := m.buf
	st := C.fs_digest_batch_multi((**C.fs_ctx)(m.ctxs), C.int(len(m.gpus)), (*C.uint8_t)(unsafe.Pointer(&buf[0])),
		C.uint64_t(len(buf)), (*C.uint64_t)(unsafe.Pointer(&g.offs[0])), (*C.uint32_t)(unsafe.Pointer(&g.lens[0])),
		C.uint32_t(n), C.uint32_t(mtu), (*C.fs_digest)(unsafe.Pointer(&out[0])),
		(*C.uint8_t)(unsafe.Pointer(&verdicts[0])))
	if st != C.FS_SUCCESS {
		for _, x := range m.gpus {
			if msg := C.GoString(C.fs_last_error(x.ctx)); msg != "" {
				return errors.New("framesum: " + msg)
			}
		}
		return errors.New("framesum: fs_digest_batch_multi failed")
	}
	return nil
}

// Group drives several GPUs of this host from one process with device-resident shards and RCCL
// (fs_group_create / fs_digest_batch_sharded; BASELINE configs[3]): frames that the NIC placed in
// the HBM of several GPUs (GPUDirect RDMA) are digested where they lie, round-robin sharded
// (global frame i is frame i / N of shard i % N; eth/crc.go:12-17: CRC791 is per call, so frames
// are independent); only the 8-byte digests and 1-byte verdicts travel, over xGMI, to the first
// device (chunk by chunk, grouped ncclSend/ncclRecv), where a de-interleave kernel restores global
// order. The consumer is the
// same as DigestBatch's: stacks.PortStack.RecvEth (stacks/portstack.go:163) -> :240 / :303.
type Group struct {
	g    *C.fs_group
	n    int
	ptrs unsafe.Pointer // C memory: frames, offsets, lengths pointer arrays of n entries each
}

// DeviceShard is shard k of a sharded batch: DEVICE pointers on the group's k-th device, laid
// out as fs_digest_batch expects (frame i = Frames[Offsets[i] : Offsets[i]+Lengths[i]]), holding
// ShardCount(n, N, k) frames. The memory is the caller's (e.g. its NIC driver's receive rings).
type DeviceShard struct {
	Frames  unsafe.Pointer // uint8
	Offsets unsafe.Pointer // uint64 per frame
	Lengths unsafe.Pointer // uint32 per frame
}

// OpenGroup creates one context, one stream and one RCCL communicator per listed device
// (distinct devices; ncclCommInitAll).
func OpenGroup(devices []int) (*Group, error) {
	if len(devices) == 0 {
		return nil, errors.New("framesum: no devices")
	}
	devs := (*C.int)(C.malloc(C.size_t(len(devices)) * C.size_t(unsafe.Sizeof(C.int(0)))))
	defer C.free(unsafe.Pointer(devs))
	arr := unsafe.Slice(devs, len(devices))
	for i, d := range devices {
		arr[i] = C.int(d)
	}
	var g *C.fs_group
	if st := C.fs_group_create(devs, C.int(len(devices)), &g); st != C.FS_SUCCESS {
		return nil, errors.New("framesum: " + C.GoString(C.fs_group_last_error(nil)))
	}
	ptrs := C.malloc(3 * C.size_t(len(devices)) * C.size_t(unsafe.Sizeof(uintptr(0))))
	return &Group{g: g, n: len(devices), ptrs: ptrs}, nil
}

// Close releases the group's contexts, streams and communicators.
func (g *Group) Close() error {
	if g.g == nil {
		return nil
	}
	C.fs_group_destroy(g.g)
	C.free(g.ptrs)
	g.g, g.ptrs = nil, nil
	return nil
}

// ShardCount is the number of frames shard `shard` holds when n global frames go round-robin
// over nshards shards (fs_shard_count).
func ShardCount(n uint64, nshards, shard int) uint64 {
	return uint64(C.fs_shard_count(C.uint64_t(n), C.uint32_t(nshards), C.uint32_t(shard)))
}

// DigestSharded digests a global batch of n frames held as one DeviceShard per group device.
// out (n Digests, 8 bytes each) and verdicts (n bytes; nil to skip) are DEVICE pointers on the
// group's first device and receive the results in global frame order. It returns when they are
// written.
func (g *Group) DigestSharded(shards []DeviceShard, n uint64, mtu uint16, out, verdicts unsafe.Pointer) error {
	if len(shards) != g.n {
		return errors.New("framesum: one DeviceShard per group device")
	}
	p := unsafe.Slice((*unsafe.Pointer)(g.ptrs), 3*g.n)
	for k, s := range shards {
		p[k], p[g.n+k], p[2*g.n+k] = s.Frames, s.Offsets, s.Lengths
	}
	st := C.fs_digest_batch_sharded(g.g, (**C.uint8_t)(unsafe.Pointer(&p[0])),
		(**C.uint64_t)(unsafe.Pointer(&p[g.n])), (**C.uint32_t)(unsafe.Pointer(&p[2*g.n])),
		C.uint64_t(n), C.uint32_t(mtu), (*C.fs_digest)(out), (*C.uint8_t)(verdicts))
	if st != C.FS_SUCCESS {
		return errors.New("framesum: " + C.GoString(C.fs_group_last_error(g.g)))
	}
	return nil
}
