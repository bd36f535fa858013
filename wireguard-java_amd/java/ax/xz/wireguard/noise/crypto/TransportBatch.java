package ax.xz.wireguard.noise.crypto;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.concurrent.ForkJoinPool;

import static java.lang.foreign.ValueLayout.*;

/**
 * The transport-data path on the MI355X: per-packet calls (what
 * SymmetricKeypair.cipher/decipher make, SymmetricKeypair.java:63-83) and the
 * batch calls a batching TransportManager makes (INTEGRATION.md §3).
 *
 * A batch is a table of 32-byte {@code wg_pkt} descriptors
 * {in_off u64, out_off u64, counter u64, len u32, key_slot u32} over one input
 * and one output buffer; seal writes ct || tag at out_off, open verifies then
 * writes pt (status[i] = 1 and a zeroed pt for a forged packet).
 */
public final class TransportBatch {
	private TransportBatch() {}

	public static int installKeys(MemorySegment sendKey, MemorySegment receiveKey) {
		return WgAead.installKeys(sendKey, receiveKey);
	}

	public static void releaseKeys(int sendSlot, int receiveSlot) {
		WgAead.releaseKeys(sendSlot, receiveSlot);
	}

	/**
	 * One blocking per-packet call. wg_seal1 / wg_open1 wait for the batched launch that
	 * carries the packet; on a ForkJoinPool worker (TransportManager.java:41 runs every
	 * packet there) the wait is a ManagedBlocker, so the pool adds workers while callers
	 * wait and more packets share each launch, without any change in ax.xz.wireguard.
	 */
	private static final class Call implements ForkJoinPool.ManagedBlocker {
		private final boolean open;
		private final int slot;
		private final long counter;
		private final MemorySegment in, out;
		private final int len;
		int rc;
		private boolean done;

		Call(boolean open, int slot, long counter, MemorySegment in, int len, MemorySegment out) {
			this.open = open;
			this.slot = slot;
			this.counter = counter;
			this.in = in;
			this.len = len;
			this.out = out;
		}

		@Override
		public boolean block() {
			try {
				rc = open ? (int) WgAead.OPEN1.invokeExact(WgAead.CTX, slot, counter, in, len, out)
				          : (int) WgAead.SEAL1.invokeExact(WgAead.CTX, slot, counter, in, len, out);
			} catch (Throwable e) {
				throw new RuntimeException(e);
			}
			done = true;
			return true;
		}

		@Override
		public boolean isReleasable() {
			return done;
		}

		int run() {
			try {
				ForkJoinPool.managedBlock(this);  // off a pool worker this just calls block()
			} catch (InterruptedException e) {
				Thread.currentThread().interrupt();
				throw new RuntimeException(e);
			}
			return WgAead.check(rc);
		}
	}

	/** dst (len + 16 bytes) = ChaCha20-Poly1305(key[slot], LE64(counter) || 0^4, src). */
	public static void seal1(int slot, long counter, MemorySegment src, MemorySegment dst) {
		try (var arena = Arena.ofConfined()) {
			var in = native_(arena, src);
			var out = dst.isNative() ? dst : arena.allocate(dst.byteSize(), 16);
			new Call(false, slot, counter, in, (int) src.byteSize(), out).run();
			if (out != dst)
				dst.copyFrom(out);
		}
	}

	/** Verify-then-decrypt src = ct || tag into dst; false (dst untouched) on a bad tag. */
	public static boolean open1(int slot, long counter, MemorySegment src, MemorySegment dst) {
		try (var arena = Arena.ofConfined()) {
			var in = native_(arena, src);
			var out = arena.allocate(Math.max(1, dst.byteSize()), 16);
			int rc = new Call(true, slot, counter, in, (int) (src.byteSize() - 16), out).run();
			if (rc != 0)
				return false;
			dst.copyFrom(out.asSlice(0, dst.byteSize()));
			return true;
		}
	}

	/** Writes descriptor {@code i} of a wg_pkt table. */
	public static void setPacket(MemorySegment table, int i, long inOff, long outOff, long counter, int len, int keySlot) {
		long b = i * WgAead.PKT_DESC_SIZE;
		table.set(JAVA_LONG, b, inOff);
		table.set(JAVA_LONG, b + 8, outOff);
		table.set(JAVA_LONG, b + 16, counter);
		table.set(JAVA_INT, b + 24, len);
		table.set(JAVA_INT, b + 28, keySlot);
	}

	/**
	 * Seals {@code n} packets whose buffers live in device memory (pointers from a
	 * device allocator); {@code stream} is the HIP stream to enqueue on (NULL: default).
	 */
	public static void sealDevice(MemorySegment table, int n, MemorySegment in, long inSize, MemorySegment out,
	                              long outSize, int maxLen, boolean uniform, MemorySegment stream) {
		try {
			WgAead.check((int) WgAead.SEAL_BATCH.invokeExact(WgAead.CTX, table, n, in, inSize, out, outSize, maxLen,
				uniform ? WgAead.WG_F_UNIFORM : 0, stream));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/** Opens {@code n} device-resident packets; status (device int32[n]) gets 0 / 1 per packet. */
	public static void openDevice(MemorySegment table, int n, MemorySegment in, long inSize, MemorySegment out,
	                              long outSize, MemorySegment status, int maxLen, boolean uniform, MemorySegment stream) {
		openDevice(table, n, in, inSize, out, outSize, status, maxLen, uniform, false, stream);
	}

	/**
	 * Opens {@code n} device-resident packets; with {@code rxFilter} (WG_F_RX_FILTER) the same launch
	 * also applies TransportManager.processDecryptedTransport's checks (TransportManager.java:98-119:
	 * keepalive, IP version, the key slot's AllowedIPs) and writes WG_PKT_KEEPALIVE / BADIP / FILTERED
	 * into {@code status} for packets that verified.
	 */
	public static void openDevice(MemorySegment table, int n, MemorySegment in, long inSize, MemorySegment out,
	                              long outSize, MemorySegment status, int maxLen, boolean uniform, boolean rxFilter,
	                              MemorySegment stream) {
		try {
			WgAead.check((int) WgAead.OPEN_BATCH.invokeExact(WgAead.CTX, table, n, in, inSize, out, outSize, status,
				maxLen, (uniform ? WgAead.WG_F_UNIFORM : 0) | (rxFilter ? WgAead.WG_F_RX_FILTER : 0), stream));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/**
	 * Seals one device-resident batch and opens another in one kernel launch (wg_duplex_batch):
	 * the node's outgoing packets (TransportManager.java:41) and its incoming ones (:79). The open
	 * batch must not read bytes the seal batch writes in the same call.
	 */
	public static void duplexDevice(MemorySegment sealTable, int nSeal, MemorySegment sealIn, long sealInSize,
	                                MemorySegment sealOut, long sealOutSize, int sealMaxLen,
	                                MemorySegment openTable, int nOpen, MemorySegment openIn, long openInSize,
	                                MemorySegment openOut, long openOutSize, MemorySegment status, int openMaxLen,
	                                boolean uniform, MemorySegment stream) {
		duplexDevice(sealTable, nSeal, sealIn, sealInSize, sealOut, sealOutSize, sealMaxLen, openTable, nOpen, openIn,
			openInSize, openOut, openOutSize, status, openMaxLen, uniform, false, stream);
	}

	/**
	 * As above; with {@code afterSeal} (WG_F_AFTER_SEAL) the open batch reads what the seal batch writes:
	 * open packet i is ordered after seal packet i (equal sizes). Uniform batches then run as one
	 * k_step launch that opens each 32-packet chunk as soon as it is sealed.
	 */
	public static void duplexDevice(MemorySegment sealTable, int nSeal, MemorySegment sealIn, long sealInSize,
	                                MemorySegment sealOut, long sealOutSize, int sealMaxLen,
	                                MemorySegment openTable, int nOpen, MemorySegment openIn, long openInSize,
	                                MemorySegment openOut, long openOutSize, MemorySegment status, int openMaxLen,
	                                boolean uniform, boolean afterSeal, MemorySegment stream) {
		try (var arena = Arena.ofConfined()) {
			var s = batch(arena, sealTable, nSeal, sealIn, sealInSize, sealOut, sealOutSize, MemorySegment.NULL,
				sealMaxLen, uniform ? WgAead.WG_F_UNIFORM : 0);
			var o = batch(arena, openTable, nOpen, openIn, openInSize, openOut, openOutSize, status, openMaxLen,
				(uniform ? WgAead.WG_F_UNIFORM : 0) | (afterSeal ? WgAead.WG_F_AFTER_SEAL : 0));
			WgAead.check((int) WgAead.DUPLEX_BATCH.invokeExact(WgAead.CTX, s, o, stream));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	// struct wg_batch {desc, in, out, status, in_size, out_size, n, max_len, flags, _reserved} (64 B)
	private static MemorySegment batch(Arena arena, MemorySegment table, int n, MemorySegment in, long inSize,
	                                   MemorySegment out, long outSize, MemorySegment status, int maxLen,
	                                   int flags) {
		var b = arena.allocate(WgAead.BATCH_SIZE, 8);
		b.set(ADDRESS, 0, table);
		b.set(ADDRESS, 8, in);
		b.set(ADDRESS, 16, out);
		b.set(ADDRESS, 24, status);
		b.set(JAVA_LONG, 32, inSize);
		b.set(JAVA_LONG, 40, outSize);
		b.set(JAVA_INT, 48, n);
		b.set(JAVA_INT, 52, maxLen);
		b.set(JAVA_INT, 56, flags);
		b.set(JAVA_INT, 60, 0);
		return b;
	}

	/**
	 * A pinned, device-mapped host ring (wg_host_alloc): packet buffers allocated here make
	 * {@link #sealHost} / {@link #openHost} zero-copy. Free with {@link #freeHostRing}.
	 */
	public static MemorySegment allocHostRing(long bytes) {
		try (var arena = Arena.ofConfined()) {
			var out = arena.allocate(ADDRESS);
			WgAead.check((int) WgAead.HOST_ALLOC.invokeExact(WgAead.CTX, bytes, out));
			return out.get(ADDRESS, 0).reinterpret(bytes);
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	public static void freeHostRing(MemorySegment ring) {
		try {
			WgAead.check((int) WgAead.HOST_FREE.invokeExact(WgAead.CTX, ring));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/** Seals a batch whose buffers are in host memory (tun ring in, UDP ring out); synchronous. */
	public static void sealHost(MemorySegment table, int n, MemorySegment in, MemorySegment out, int maxLen,
	                            boolean uniform) {
		try {
			WgAead.check((int) WgAead.SEAL_HOST.invokeExact(WgAead.CTX, table, n, in, in.byteSize(), out,
				out.byteSize(), maxLen, uniform ? WgAead.WG_F_UNIFORM : 0));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/** Opens a host-memory batch; status (int32[n], host) gets WG_PKT_OK / WG_PKT_BADTAG per packet. */
	public static void openHost(MemorySegment table, int n, MemorySegment in, MemorySegment out, MemorySegment status,
	                            int maxLen, boolean uniform) {
		try {
			WgAead.check((int) WgAead.OPEN_HOST.invokeExact(WgAead.CTX, table, n, in, in.byteSize(), out,
				out.byteSize(), status, maxLen, uniform ? WgAead.WG_F_UNIFORM : 0));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/**
	 * An AllowedIPs filter from subnets, built as IPFilter.insert builds its trie
	 * (util/IPFilter.java:30-42) and searched with IPFilter.search's rule on the device.
	 * {@code filterId} is the peer's; map the peer's receive key slots to it with {@link #mapSlots}.
	 */
	public static void setFilter(int filterId, java.net.InetAddress[] subnets, int[] prefixLengths) {
		if (subnets.length != prefixLengths.length)
			throw new IllegalArgumentException("one prefix length per subnet");
		try (var arena = Arena.ofConfined()) {
			var table = arena.allocate(18L * Math.max(1, subnets.length), 1);  // wg_prefix {u8 family, u8 len, u8 addr[16]}
			for (int i = 0; i < subnets.length; i++) {
				byte[] a = subnets[i].getAddress();
				table.set(JAVA_BYTE, 18L * i, (byte) (a.length == 4 ? 4 : 6));
				table.set(JAVA_BYTE, 18L * i + 1, (byte) prefixLengths[i]);
				MemorySegment.copy(MemorySegment.ofArray(a), 0, table, 18L * i + 2, a.length);
			}
			WgAead.check((int) WgAead.FILTER_SET.invokeExact(WgAead.CTX, filterId, table, subnets.length));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/** Filter id per key slot for slots [first, first + ids.length); WgAead.WG_NO_FILTER = pass all. */
	public static void mapSlots(int firstSlot, int[] ids) {
		try (var arena = Arena.ofConfined()) {
			var a = arena.allocate(4L * Math.max(1, ids.length), 4);
			MemorySegment.copy(MemorySegment.ofArray(ids), 0, a, 0, 4L * ids.length);
			WgAead.check((int) WgAead.SLOT_FILTERS_SET.invokeExact(WgAead.CTX, firstSlot, ids.length, a));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/** Per-key-slot replay window of {@code windowBits} (the reference has none); 0 disables. */
	public static void enableReplayWindow(int windowBits) {
		try {
			WgAead.check((int) WgAead.REPLAY_ENABLE.invokeExact(WgAead.CTX, windowBits));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/**
	 * processDecryptedTransport for an opened device batch (run after {@link #openDevice} on
	 * the same stream): status[i] stays WG_PKT_OK (forward to the tun queue) or becomes
	 * WG_PKT_KEEPALIVE / WG_PKT_BADIP / WG_PKT_FILTERED / WG_PKT_REPLAY (drop).
	 */
	public static void rxCheck(MemorySegment table, int n, MemorySegment pt, long ptSize, MemorySegment status,
	                           int flags, MemorySegment stream) {
		try {
			WgAead.check((int) WgAead.RX_CHECK.invokeExact(WgAead.CTX, table, n, pt, ptSize, status, flags, stream));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	public static void sync(MemorySegment stream) {
		try {
			WgAead.check((int) WgAead.SYNC.invokeExact(WgAead.CTX, stream));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	private static MemorySegment native_(Arena arena, MemorySegment s) {
		return s.isNative() ? s : arena.allocate(Math.max(1, s.byteSize()), 16).copyFrom(s);
	}
}
