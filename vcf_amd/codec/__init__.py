"""The reference's plug-in surface, composed explicitly.

    parser   -- the CLI options of parser.py / 2D-DCT.py / YCoCg.py /
                deadzone.py / no_filter.py / entropy_image_coding.py / III.py
    eic      -- entropy_image_coding.CoDec file I/O
    tiff     -- TIFF.CoDec (byte-exact tifffile 2021.7.2 writer, reader)
    dct2d    -- 2D-DCT.CoDec (encode_fn/decode_fn; the hot span on the GPU)
    iii      -- III.CoDec (frame loop, sharded one process per GPU)
    shard    -- frame partitioning and the size/payload exchange
    main     -- main.main
Submodules import lazily; nothing here touches the GPU at import time.
"""
