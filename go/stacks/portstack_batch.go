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
	"errors"
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

// errUnexpectedVerdict: a frame reached the delivery step with a verdict that is not
// VerdictOK and that no earlier step ends the frame on (VerdictFCS, a value this file does not
// know, a corrupted status byte). Such a frame is never handed to a socket: fail closed.
var errUnexpectedVerdict = errors.New("stacks: RecvEthBatch: unexpected GPU verdict")

// gateKind is one step of RecvEth's decision order (portstack.go:163-355) once the GPU has
// evaluated a frame's byte-level gates. recvEthVerified walks recvEthGates in order; the order
// and the verdict classes each step ends the frame on are data, so that
// tests/test_go_gate_order.py reads this table from this file and checks it, for every verdict
// and every stack state (MAC filter, IP filter, open sockets), against a transliteration of
// RecvEth's branches.
type gateKind uint8

const (
	gateLength    gateKind = iota // :167-172 frame length < 34 -> errPacketSmol; > MTU -> errPacketExceedsMTU
	gateGlobal                    // :178-184 the stack's global handler (its error ends the frame)
	gateMAC                       // :186-187 destination MAC neither broadcast nor ours -> nil
	gateEtherType                 // :187-197 not IPv4 or ARP -> nil; ARP: length gate, then the ARP client
	gateVerdict                   // the GPU verdict ends the frame when it is one of the step's classes
	gateIPDest                    // :209-210 IP destination neither ours nor our address unset -> nil
	gateSockets                   // :223, :284 no socket of the frame's protocol -> nil
	gateDeliver                   // :246-281 UDP, :309-346 TCP: the segment to its port's handler
)

type gate struct {
	kind    gateKind
	classes []eth.Verdict // gateVerdict: the verdicts that end the frame at this step
	logged  bool          // gateVerdict: RecvEth logs the error (the protocol switch, :348-350)
}

// recvEthGates is RecvEth's branch order (portstack.go:163-355) around the GPU verdict.
var recvEthGates = [...]gate{
	{kind: gateLength},
	{kind: gateGlobal},
	{kind: gateMAC},
	{kind: gateEtherType},
	{kind: gateVerdict, classes: []eth.Verdict{eth.VerdictIPVersion, eth.VerdictInvalidIHL}},
	{kind: gateIPDest},
	{kind: gateVerdict, classes: []eth.Verdict{eth.VerdictBadIPTotalLenOrIHL, eth.VerdictExceedsMTU}},
	{kind: gateVerdict, classes: []eth.Verdict{eth.VerdictUnknownIPProto}, logged: true},
	{kind: gateSockets},
	{kind: gateVerdict, classes: []eth.Verdict{eth.VerdictTooShortTCPOrUDP, eth.VerdictZeroPort, eth.VerdictBadUDPLength, eth.VerdictBadTCPOffset, eth.VerdictChecksum}, logged: true},
	{kind: gateDeliver},
}

// recvEthVerified finishes one frame whose byte-level gates and L4 checksum the GPU has
// evaluated (verdict v). The GPU applies RecvEth's gates in RecvEth's order under a fixed
// stack model (no MAC / IP destination filter, sockets open); the steps of recvEthGates put
// the stack-state branches back at the point where RecvEth takes them, so a verdict only
// counts once the frame has got that far.
func (ps *PortStack) recvEthVerified(frame []byte, v eth.Verdict) error {
	var (
		ehdr     *eth.EthernetHeader
		ihdr     eth.IPv4Header
		ipOffset uint8
	)
	for _, g := range recvEthGates {
		switch g.kind {
		case gateLength:
			if len(frame) < eth.SizeEthernetHeader+eth.SizeIPv4Header {
				return errPacketSmol
			} else if len(frame) > int(ps.mtu) {
				return errPacketExceedsMTU
			}
			ps.trace("Stack.RecvEth:start", slog.Int("plen", len(frame)))
			ps.lastRx = ps.now()
			ps.auxEth = eth.DecodeEthernetHeader(frame)
			ehdr = &ps.auxEth
		case gateGlobal:
			if ps.glob != nil {
				if err := ps.glob(ehdr, frame[eth.SizeEthernetHeader:]); err != nil {
					return err
				}
			}
		case gateMAC:
			if ehdr.Destination != eth.BroadcastHW6() && ehdr.Destination != ps.mac {
				return nil
			}
		case gateEtherType:
			switch ehdr.AssertType() {
			case eth.EtherTypeARP:
				if v == eth.VerdictPacketSmol { // the ARP length gate (:192-194)
					return errPacketSmol
				}
				ps.auxARP = eth.DecodeARPv4Header(frame[eth.SizeEthernetHeader:])
				return ps.arpClient.recv(&ps.auxARP)
			case eth.EtherTypeIPv4:
				ihdr, ipOffset = eth.DecodeIPv4Header(frame[eth.SizeEthernetHeader:])
			default:
				return nil
			}
		case gateVerdict:
			for _, c := range g.classes {
				if v == c {
					err := verdictErr[v]
					if g.logged && err != nil {
						ps.error("Stack.RecvEth", slog.String("err", err.Error()))
					}
					return err
				}
			}
		case gateIPDest:
			if ps.ip != ihdr.Destination && ps.ip != [4]byte{} {
				return nil
			}
		case gateSockets:
			if (ihdr.Protocol == 17 && len(ps.portsUDP) == 0) || (ihdr.Protocol == 6 && len(ps.portsTCP) == 0) {
				return nil // RecvEth stops before its L4 gates
			}
		case gateDeliver:
			if v != eth.VerdictOK { // fail closed: only a verified frame reaches a socket
				return errUnexpectedVerdict
			}
			offset := eth.SizeEthernetHeader + int(ipOffset)
			segment := frame[offset : eth.SizeEthernetHeader+int(ihdr.TotalLength)]
			var err error
			if ihdr.Protocol == 17 {
				err = ps.deliverUDP(ehdr, &ihdr, segment)
			} else {
				err = ps.deliverTCP(ehdr, &ihdr, frame[eth.SizeEthernetHeader+eth.SizeIPv4Header:offset], segment)
			}
			if err != nil {
				ps.error("Stack.RecvEth", slog.String("err", err.Error()))
			}
			return err
		}
	}
	return nil
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
