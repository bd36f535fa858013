package ax.xz.wireguard.noise.crypto;

import java.io.ByteArrayOutputStream;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;

import static java.lang.foreign.ValueLayout.JAVA_BYTE;

/**
 * Drop-in for ax.xz.wireguard.noise.crypto.Poly1305 (reference Poly1305.java):
 * init / update / finish with the same state errors. Updates are buffered and the
 * one-shot MAC (wg_aead_host, WG_MODE_MAC) runs at finish — the same tag as
 * donna's streaming update (poly1305-donna.c:26-61).
 */
public class Poly1305 {
	private final ByteArrayOutputStream buffer = new ByteArrayOutputStream();
	private byte[] key;
	private boolean finished = false, initialised = false;

	Poly1305(Arena arena) {}

	Poly1305(MemorySegment context) {}

	public Poly1305() {}

	public void init(MemorySegment key) {
		this.key = key.asSlice(0, 32).toArray(JAVA_BYTE);
		buffer.reset();
		initialised = true;
		finished = false;
	}

	public void update(MemorySegment message) {
		if (finished)
			throw new IllegalStateException("Poly1305 context has already been finished");
		if (!initialised)
			throw new IllegalStateException("Poly1305 context has not been initialised");
		buffer.writeBytes(message.toArray(JAVA_BYTE));
	}

	public void finish(MemorySegment mac) {
		if (finished)
			throw new IllegalStateException("Poly1305 context has already been finished");
		if (!initialised)
			throw new IllegalStateException("Poly1305 context has not been initialised");
		byte[] msg = buffer.toByteArray();
		WgAead.aead(WgAead.WG_MODE_MAC, MemorySegment.ofArray(key), 0, 0, 0, 0, MemorySegment.ofArray(msg), null,
			mac.asSlice(0, 16), msg.length);
		java.util.Arrays.fill(key, (byte) 0);
		finished = true;
	}

	public byte[] finish() {
		try (var arena = Arena.ofConfined()) {
			var mac = arena.allocate(16, 1);
			finish(mac);
			return mac.toArray(JAVA_BYTE);
		}
	}
}
