//go:build framesum

// Package stacks addition: RecvEthBatch, the batched receive path over the framesum
// GPU engine (SURVEY.md §8f rank 3). Drop next to portstack.go in soypat/seqs/stacks/
// together with eth/digest_gpu.go and build with `-tags framesum`.
//
// RecvEth (portstack.go:163-355) does, per frame, O(1) header work and one O(len) scan:
// the L4 checksum (CalculateChecksumIPv4 at :239 / :303, the CRC791 loop of eth/crc.go).
// RecvEthBatch moves that scan, and every gate that only depends on the frame's bytes,
// to the GPU for a whole batch in one call (eth.GPU.DigestBatch), then finishes each
// frame here with the parts that depend on the stack's own state: the global handler,
// the MAC and IP destination filters, whether sockets are open, and the delivery to the
// port's handler. errs[i] is what RecvEth(frames[i]) returns, frame for frame, and the
// stack's side effects are the same as for RecvEth called on the frames in order.
package stacks

import (
	"io"
	"log/slog"

	"github.com/soypat/seqs/eth"
)

// EthBatch holds a GPU context and the per-batch result buffers RecvEthBatch reuses.
type EthBatch struct {
	gpu *eth.GPU
	dig []eth.Digest
	ver []eth.Verdict
}

// NewEthBatch wraps an open GPU context (eth.OpenGPU) for RecvEthBatch.
func NewEthBatch(g *eth.GPU) *EthBatch { return &EthBatch{gpu: g} }

// RecvEthBatch receives a batch of Ethernet frames. The GPU digests the batch with the
// stack's MTU; then each frame is finished in batch order. errs must hold len(frames);
// the returned error is the GPU call's own failure (then no frame was received).
func (ps *PortStack) RecvEthBatch(b *EthBatch, frames [][]byte, errs []error) error {
	n := len(frames)
	if cap(b.dig) < n {
		b.dig = make([]eth.Digest, n)
		b.ver = make([]eth.Verdict, n)
	}
	dig, ver := b.dig[:n], b.ver[:n]
	if err := b.gpu.DigestBatch(frames, ps.mtu, dig, ver); err != nil {
		return err
	}
	for i, f := range frames {
		errs[i] = ps.recvEthVerified(f, ver[i])
	}
	return nil
}

// verdictErr: the RecvEth error of each fs_verdict (portstack.go:120-142); nil for the
// classes RecvEth ignores.
var verdictErr = [...]error{
	eth.VerdictOK:                 nil,
	eth.VerdictPacketSmol:         errPacketSmol,
	eth.VerdictExceedsMTU:         errPacketExceedsMTU,
	eth.VerdictNotIPv4:            nil,
	eth.VerdictARP:                nil,
	eth.VerdictIPVersion:          errIPVersion,
	eth.VerdictInvalidIHL:         errInvalidIHL,
	eth.VerdictBadIPTotalLenOrIHL: errBadIPTotalLenOrIHL,
	eth.VerdictUnknownIPProto:     errUnknownIPProto,
	eth.VerdictTooShortTCPOrUDP:   errTooShortTCPOrUDP,
	eth.VerdictZeroPort:           errZeroPort,
	eth.VerdictBadUDPLength:       errBadUDPLength,
	eth.VerdictBadTCPOffset:       errBadTCPOffset,
	eth.VerdictChecksum:           ErrChecksumTCPorUDP,
}

// recvEthVerified finishes one frame whose byte-level gates and L4 checksum the GPU has
// evaluated (verdict v). The GPU applies RecvEth's gates in RecvEth's order under a fixed
// stack model (no MAC / IP destination filter, sockets open); here the stack-state
// branches are put back at the point where RecvEth takes them, so a verdict only counts
// once the frame has got that far.
func (ps *PortStack) recvEthVerified(frame []byte, v eth.Verdict) error {
	// The length gates come before anything else (:167-172).
	if len(frame) < eth.SizeEthernetHeader+eth.SizeIPv4Header {
		return errPacketSmol
	} else if len(frame) > int(ps.mtu) {
		return errPacketExceedsMTU
	}
	ps.trace("Stack.RecvEth:start", slog.Int("plen", len(frame)))
	ps.lastRx = ps.now()
	ps.auxEth = eth.DecodeEthernetHeader(frame)
	ehdr := &ps.auxEth
	if ps.glob != nil {
		if err := ps.glob(ehdr, frame[eth.SizeEthernetHeader:]); err != nil {
			return err
		}
	}
	// Destination MAC and EtherType filters (:185-189).
	if ehdr.Destination != eth.BroadcastHW6() && ehdr.Destination != ps.mac {
		return nil
	}
	switch ehdr.AssertType() {
	case eth.EtherTypeARP: // (:191-197) the only gate is the ARP length
		if v == eth.VerdictPacketSmol {
			return errPacketSmol
		}
		ps.auxARP = eth.DecodeARPv4Header(frame[eth.SizeEthernetHeader:])
		return ps.arpClient.recv(&ps.auxARP)
	case eth.EtherTypeIPv4:
	default:
		return nil
	}
	ihdr, ipOffset := eth.DecodeIPv4Header(frame[eth.SizeEthernetHeader:])
	// Version and IHL come before the IP destination filter, the length and MTU gates after
	// it (:203-215).
	if v == eth.VerdictIPVersion || v == eth.VerdictInvalidIHL {
		return verdictErr[v]
	}
	if ps.ip != ihdr.Destination && ps.ip != [4]byte{} {
		return nil
	}
	if v == eth.VerdictBadIPTotalLenOrIHL || v == eth.VerdictExceedsMTU {
		return verdictErr[v]
	}
	// The protocol switch (:218-347): its errors are the ones RecvEth logs.
	var err error
	switch {
	case v == eth.VerdictUnknownIPProto:
		err = verdictErr[v]
	case (ihdr.Protocol == 17 && len(ps.portsUDP) == 0) || (ihdr.Protocol == 6 && len(ps.portsTCP) == 0):
		// no socket of the frame's protocol: RecvEth stops before its L4 gates (:223, :284)
	case v != eth.VerdictOK:
		err = verdictErr[v]
	default: // verified: hand the segment to its socket (:246-281 UDP, :309-346 TCP)
		offset := eth.SizeEthernetHeader + int(ipOffset)
		segment := frame[offset : eth.SizeEthernetHeader+int(ihdr.TotalLength)]
		if ihdr.Protocol == 17 {
			err = ps.deliverUDP(ehdr, &ihdr, segment)
		} else {
			err = ps.deliverTCP(ehdr, &ihdr, frame[eth.SizeEthernetHeader+eth.SizeIPv4Header:offset], segment)
		}
	}
	if err != nil {
		ps.error("Stack.RecvEth", slog.String("err", err.Error()))
	}
	return err
}

// deliverUDP passes a verified UDP datagram to the port listening on its destination port.
func (ps *PortStack) deliverUDP(ehdr *eth.EthernetHeader, ihdr *eth.IPv4Header, segment []byte) error {
	uhdr := eth.DecodeUDPHeader(segment)
	port := findPort(ps.portsUDP, uhdr.DestinationPort)
	if port == nil {
		return nil
	}
	payload := segment[eth.SizeUDPHeader:]
	if ps.isLogEnabled(slog.LevelDebug) {
		ps.debug("UDP:recv", slog.Int("plen", len(payload)))
	}
	ps.pendingUDPv4++
	pkt := &ps.auxUDP
	pkt.Rx, pkt.Eth, pkt.IP, pkt.UDP = ps.lastRx, *ehdr, *ihdr, uhdr
	copy(pkt.payload[:], payload)
	return ps.settle(port.ihandler.recv(pkt), port.Close)
}

// deliverTCP passes a verified TCP segment (IP options, TCP options and payload, in that
// order in the packet's data) to the port listening on its destination port.
func (ps *PortStack) deliverTCP(ehdr *eth.EthernetHeader, ihdr *eth.IPv4Header, ipOptions, segment []byte) error {
	thdr, off := eth.DecodeTCPHeader(segment)
	port := findPort(ps.portsTCP, thdr.DestinationPort)
	if port == nil {
		if ps.isLogEnabled(slog.LevelDebug) {
			ps.debug("tcp:noSocket", slog.Int("port", int(thdr.DestinationPort)), slog.Int("avail", len(ps.portsTCP)))
		}
		return nil
	}
	tcpOptions, payload := segment[eth.SizeTCPHeader:off], segment[off:]
	if ps.isLogEnabled(slog.LevelDebug) {
		ps.debug("TCP:recv", slog.Int("opt", len(tcpOptions)), slog.Int("ipopt", len(ipOptions)),
			slog.Int("payload", len(payload)))
	}
	ps.pendingTCPv4++
	pkt := &ps.auxTCP
	pkt.Rx, pkt.Eth, pkt.IP, pkt.TCP = ps.lastRx, *ehdr, *ihdr, thdr
	k := copy(pkt.data[:], ipOptions)
	k += copy(pkt.data[k:], tcpOptions)
	copy(pkt.data[k:], payload)
	return ps.settle(port.handler.recv(pkt), port.Close)
}

// settle maps a handler's return as RecvEth does: io.EOF closes the port, ErrFlagPending
// is not an error.
func (ps *PortStack) settle(err error, closePort func()) error {
	switch err {
	case io.EOF:
		closePort()
		return nil
	case ErrFlagPending:
		return nil
	}
	return err
}
