package ax.xz.wireguard.noise.crypto;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.util.concurrent.ConcurrentLinkedDeque;

import static java.lang.foreign.ValueLayout.*;

/**
 * Panama (FFM) binding of libwgaead.so — the MI355X transport AEAD (include/wgaead.h).
 *
 * Replaces the two downcall libraries the reference binds today:
 * libchacha (ChaCha20.java:14-42) and libpoly1305-donna (Poly1305.java:24-77).
 * Same conventions: the library is found through -Djava.library.path
 * (run.sh:4), a known-answer self test runs at class initialisation and an
 * {@link ExceptionInInitializerError} is thrown if it fails (Poly1305.java:62-76).
 *
 * Only API present in both JDK 21 (--enable-preview, as the reference builds)
 * and JDK 22+ is used.
 */
public final class WgAead {
	public static final int WG_OK = 0;
	public static final int WG_MODE_SEAL = 0, WG_MODE_OPEN = 1, WG_MODE_CIPHER = 2, WG_MODE_MAC = 3;
	public static final int WG_F_UNIFORM = 1;
	public static final int WG_F_FRAME = 2;
	public static final int WG_F_AFTER_SEAL = 4;
	public static final int WG_F_RX_FILTER = 8;
	public static final int WG_PKT_OK = 0, WG_PKT_BADTAG = 1, WG_PKT_BADHDR = 2;
	/** wg_rx_check outcomes (TransportManager.processDecryptedTransport, TransportManager.java:98-119). */
	public static final int WG_PKT_KEEPALIVE = 3, WG_PKT_BADIP = 4, WG_PKT_FILTERED = 5, WG_PKT_REPLAY = 6;
	public static final int WG_RX_FILTER = 1, WG_RX_REPLAY = 2, WG_NO_FILTER = -1;
	public static final long AEAD_DESC_SIZE = 64, PKT_DESC_SIZE = 32, BATCH_SIZE = 64;

	static final MethodHandle SELFTEST, CTX_CREATE, LAST_ERROR, KEYS_SET, KEYS_ZERO, SEAL1, OPEN1, AEAD_HOST,
		SEAL_BATCH, OPEN_BATCH, SYNC, SEAL_HOST, OPEN_HOST, HOST_ALLOC, HOST_FREE, FRAME_SEAL, PARSE_OPEN,
		FILTER_SET, SLOT_FILTERS_SET, REPLAY_ENABLE, REPLAY_RESET, RX_CHECK, DUPLEX_BATCH, QUEUE_CREATE,
		QUEUE_DESTROY, SUBMIT_SEAL, SUBMIT_OPEN, SUBMIT_SEAL_N, SUBMIT_OPEN_N, REAP, REAP_DONE, QUEUE_SUBMIT_TIMEOUT,
		NUMA_NODE;

	/** The process-wide context (one HIP device, its stream and its device key table). */
	static final MemorySegment CTX;
	static final int KEY_SLOTS;
	private static final ConcurrentLinkedDeque<Integer> FREE_SLOTS = new ConcurrentLinkedDeque<>();

	static {
		System.loadLibrary("wgaead");
		var symbols = SymbolLookup.loaderLookup();
		var linker = Linker.nativeLinker();
		SELFTEST = down(linker, symbols, "wg_aead_selftest", FunctionDescriptor.of(JAVA_INT, JAVA_INT));
		CTX_CREATE = down(linker, symbols, "wg_ctx_create", FunctionDescriptor.of(JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS));
		LAST_ERROR = down(linker, symbols, "wg_last_error", FunctionDescriptor.of(ADDRESS));
		KEYS_SET = down(linker, symbols, "wg_keys_set", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS));
		KEYS_ZERO = down(linker, symbols, "wg_keys_zero", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT));
		SEAL1 = down(linker, symbols, "wg_seal1",
			FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG, ADDRESS, JAVA_INT, ADDRESS));
		OPEN1 = down(linker, symbols, "wg_open1",
			FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG, ADDRESS, JAVA_INT, ADDRESS));
		AEAD_HOST = down(linker, symbols, "wg_aead_host", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS,
			JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
		SEAL_BATCH = down(linker, symbols, "wg_seal_batch", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT,
			ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, JAVA_INT, JAVA_INT, ADDRESS));
		OPEN_BATCH = down(linker, symbols, "wg_open_batch", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT,
			ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS));
		SYNC = down(linker, symbols, "wg_sync", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
		// device-side wire framing (TransportPacket.java:18-35): header write on seal, header parse on open
		FRAME_SEAL = down(linker, symbols, "wg_frame_seal", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT,
			ADDRESS, ADDRESS, JAVA_LONG, JAVA_LONG, JAVA_INT, ADDRESS));
		PARSE_OPEN = down(linker, symbols, "wg_parse_open", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG,
			ADDRESS, ADDRESS, ADDRESS, JAVA_INT, ADDRESS, ADDRESS, ADDRESS));
		SEAL_HOST = down(linker, symbols, "wg_seal_host", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT,
			ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, JAVA_INT, JAVA_INT));
		OPEN_HOST = down(linker, symbols, "wg_open_host", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT,
			ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS, JAVA_INT, JAVA_INT));
		HOST_ALLOC = down(linker, symbols, "wg_host_alloc", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS));
		HOST_FREE = down(linker, symbols, "wg_host_free", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
		// receive side after open (TransportManager.java:98-130, util/IPFilter.java)
		FILTER_SET = down(linker, symbols, "wg_filter_set", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS,
			JAVA_INT));
		SLOT_FILTERS_SET = down(linker, symbols, "wg_slot_filters_set", FunctionDescriptor.of(JAVA_INT, ADDRESS,
			JAVA_INT, JAVA_INT, ADDRESS));
		REPLAY_ENABLE = down(linker, symbols, "wg_replay_enable", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
		REPLAY_RESET = down(linker, symbols, "wg_replay_reset", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT,
			JAVA_INT));
		RX_CHECK = down(linker, symbols, "wg_rx_check", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT,
			ADDRESS, JAVA_LONG, ADDRESS, JAVA_INT, ADDRESS));
		// outgoing seal + incoming open in one launch (two wg_batch structs of 64 bytes)
		DUPLEX_BATCH = down(linker, symbols, "wg_duplex_batch", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS,
			ADDRESS));

		// asynchronous batch submission (TransportQueue: TransportManager.java:41,70-93,137-158)
		QUEUE_CREATE = down(linker, symbols, "wg_queue_create", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT,
			JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS));
		QUEUE_DESTROY = down(linker, symbols, "wg_queue_destroy", FunctionDescriptor.of(JAVA_INT, ADDRESS));
		SUBMIT_SEAL = down(linker, symbols, "wg_submit_seal", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT,
			JAVA_LONG, ADDRESS, JAVA_INT, JAVA_LONG));
		SUBMIT_OPEN = down(linker, symbols, "wg_submit_open", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT,
			JAVA_LONG, ADDRESS, JAVA_INT, JAVA_LONG));
		SUBMIT_SEAL_N = down(linker, symbols, "wg_submit_seal_n", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS,
			JAVA_INT));
		SUBMIT_OPEN_N = down(linker, symbols, "wg_submit_open_n", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS,
			JAVA_INT));
		REAP = down(linker, symbols, "wg_reap", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, JAVA_INT));
		REAP_DONE = down(linker, symbols, "wg_reap_done", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT));
		QUEUE_SUBMIT_TIMEOUT = down(linker, symbols, "wg_queue_set_submit_timeout", FunctionDescriptor.of(JAVA_INT,
			ADDRESS, JAVA_INT));
		// where to place the threads that feed the GPU (a queue's dispatcher already runs there)
		NUMA_NODE = down(linker, symbols, "wg_device_numa_node", FunctionDescriptor.of(JAVA_INT, JAVA_INT));

		int device = Integer.getInteger("wg.device", 0);
		KEY_SLOTS = Integer.getInteger("wg.keySlots", 65536);
		try {
			if ((int) SELFTEST.invokeExact(device) != 1)
				throw new ExceptionInInitializerError("wgaead self-test failed");
			try (var arena = Arena.ofConfined()) {
				var out = arena.allocate(ADDRESS);
				check((int) CTX_CREATE.invokeExact(device, KEY_SLOTS, out));
				CTX = out.get(ADDRESS, 0);
			}
		} catch (Throwable e) {
			throw new ExceptionInInitializerError(e);
		}
		for (int i = 0; i < KEY_SLOTS; i++)
			FREE_SLOTS.add(i);
	}

	private WgAead() {}

	/**
	 * NUMA node of the GPU (-1 if unknown): TransportManager's pools are best started on its CPUs
	 * (numactl --cpunodebind, or a thread factory that sets the affinity), as the queue's
	 * dispatcher thread is.
	 */
	public static int numaNode() {
		try {
			return (int) NUMA_NODE.invokeExact(Integer.getInteger("wg.device", 0));
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	private static MethodHandle down(Linker linker, SymbolLookup symbols, String name, FunctionDescriptor fd) {
		return symbols.find(name).map(addr -> linker.downcallHandle(addr, fd)).orElseThrow();
	}

	/** include/wgaead.h WG_ENOKEY: a per-packet call or queue submit on a key slot without a key. */
	static final int WG_ENOKEY = -126;

	/** Negative return codes become RuntimeExceptions, as the reference's wrappers do (ChaCha20.java:102,110,141). */
	static int check(int rc) {
		if (rc < 0) {
			String msg;
			try {
				var p = ((MemorySegment) LAST_ERROR.invokeExact()).reinterpret(4096);
				var sb = new StringBuilder();
				for (long i = 0; i < 4096 && p.get(JAVA_BYTE, i) != 0; i++)
					sb.append((char) p.get(JAVA_BYTE, i));
				msg = sb.toString();
			} catch (Throwable t) {
				msg = "";
			}
			// WG_ENOKEY: the key slot was zeroed (clean()) or never set; the reference's cipher() / decipher()
			// on a cleaned keypair fail on its closed key arena with an IllegalStateException
			if (rc == WG_ENOKEY)
				throw new IllegalStateException("libwgaead: key slot without a key (keypair cleaned): " + msg);
			throw new RuntimeException("libwgaead error " + rc + ": " + msg);
		}
		return rc;
	}

	/** Claims two consecutive device key slots and uploads send || receive keys. */
	static int installKeys(MemorySegment sendKey, MemorySegment receiveKey) {
		Integer a = FREE_SLOTS.pollFirst();
		Integer b = FREE_SLOTS.pollFirst();
		if (a == null || b == null)
			throw new RuntimeException("device key table full");
		try (var arena = Arena.ofConfined()) {
			var k = arena.allocate(32, 16);
			k.copyFrom(sendKey.asSlice(0, 32));
			check((int) KEYS_SET.invokeExact(CTX, (int) a, 1, k));
			k.copyFrom(receiveKey.asSlice(0, 32));
			check((int) KEYS_SET.invokeExact(CTX, (int) b, 1, k));
			k.fill((byte) 0);
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
		return (a << 16) | b;
	}

	/**
	 * SymmetricKeypair.clean: zero both device key slots and release them (SymmetricKeypair.java:85-93).
	 * Called once per keypair (its Cleanable); a slot that is already free is not released again.
	 */
	static void releaseKeys(int send, int receive) {
		if (FREE_SLOTS.contains(send) || FREE_SLOTS.contains(receive))
			throw new IllegalStateException("key slots " + send + "/" + receive + " released twice");
		try {
			check((int) KEYS_ZERO.invokeExact(CTX, send, 1));
			check((int) KEYS_ZERO.invokeExact(CTX, receive, 1));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
		FREE_SLOTS.add(send);
		FREE_SLOTS.add(receive);
	}

	/**
	 * One general AEAD / primitive call on host buffers (wg_aead_host).
	 * Returns the per-packet status of an OPEN (WG_PKT_OK / WG_PKT_BADTAG).
	 */
	static int aead(int mode, MemorySegment key, int nonce0, int nonce1, int nonce2, int ctr0, MemorySegment in,
	                MemorySegment aad, MemorySegment out, long len) {
		try (var arena = Arena.ofConfined()) {
			var desc = arena.allocate(AEAD_DESC_SIZE, 16);
			desc.set(JAVA_LONG, 0, 0L);              // in_off
			desc.set(JAVA_LONG, 8, 0L);              // out_off
			desc.set(JAVA_LONG, 16, 0L);             // aad_off
			desc.set(JAVA_INT, 24, (int) len);       // len
			desc.set(JAVA_INT, 28, aad == null ? 0 : (int) aad.byteSize());
			desc.set(JAVA_INT, 32, 0);               // key_slot
			desc.set(JAVA_INT, 36, ctr0);
			desc.set(JAVA_INT, 40, nonce0);
			desc.set(JAVA_INT, 44, nonce1);
			desc.set(JAVA_INT, 48, nonce2);
			var k = arena.allocate(32, 16).copyFrom(key.asSlice(0, 32));
			var status = arena.allocate(JAVA_INT);
			MemorySegment inN = in == null ? MemorySegment.NULL : native_(arena, in);
			MemorySegment aadN = aad == null ? MemorySegment.NULL : native_(arena, aad);
			var outN = out.isNative() ? out : arena.allocate(out.byteSize(), 16);
			check((int) AEAD_HOST.invokeExact(CTX, mode, desc, 1, k, 1, inN, in == null ? 0L : in.byteSize(), aadN,
				aad == null ? 0L : aad.byteSize(), outN, out.byteSize(), status));
			k.fill((byte) 0);
			if (outN != out)
				out.copyFrom(outN);
			return status.get(JAVA_INT, 0);
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
