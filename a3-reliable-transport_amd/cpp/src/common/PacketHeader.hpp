// PacketHeader.hpp — WTP wire header, byte-identical to the reference's
// cpp/src/common/PacketHeader.hpp:5-10: four host-order u32 in memory, each htonl'd on
// the wire (cpp/src/base/Packet.cpp:40-47) and ntohl'd on parse (Receiver.cpp:27-30).
#pragma once

#include <arpa/inet.h>

#include <cstdint>
#include <cstring>

struct PacketHeader {
    uint32_t type;      // 0 START, 1 END, 2 DATA, 3 ACK (cpp/src/base/Packet.hpp:8-13)
    uint32_t seqNum;
    uint32_t length;    // payload bytes; 0 for ACK
    uint32_t checksum;  // CRC-32 of the payload only (README.md:64)
};
static_assert(sizeof(PacketHeader) == 16, "WTP header must stay 16 bytes");

namespace wtp {

enum PacketType : uint32_t { START = 0, END = 1, DATA = 2, ACK = 3 };
constexpr size_t kHeaderBytes = sizeof(PacketHeader);
constexpr size_t kMaxPayload = 1456;  // 1500 - 20 (IP) - 8 (UDP) - 16 (header)
constexpr size_t kMaxDatagram = kHeaderBytes + kMaxPayload;

inline void put_header(uint8_t *wire, const PacketHeader &h) {
    const uint32_t be[4] = {htonl(h.type), htonl(h.seqNum), htonl(h.length), htonl(h.checksum)};
    std::memcpy(wire, be, sizeof be);
}

inline PacketHeader get_header(const uint8_t *wire) {
    uint32_t be[4];
    std::memcpy(be, wire, sizeof be);
    return PacketHeader{ntohl(be[0]), ntohl(be[1]), ntohl(be[2]), ntohl(be[3])};
}

}  // namespace wtp
